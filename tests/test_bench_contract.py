"""bench.py driver contract on the multi-rank path: 2 gloo ranks under torch.distributed.run on the CPU print ONE
JSON line with the whole-job value, world size 2, the engine's collectives, and a parity-checked baseline."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_bench_two_rank_gloo_contract(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--ring-mb", "8"]
    res = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=580)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2 * 8192
    assert out["dist"]["world_size_seen"] == 2 and out["dist"]["backend"] == "gloo"
    assert out["dist"]["engine_collectives"]["all_reduce"] >= 1
    assert out["value"] > 0 and out["vs_baseline"] is not None and out["higher_is_better"] is True


def _self_launch(tmp_path, script, *args, extra_env=None):
    """``python <script> --gpus 2 ...`` WITHOUT torchrun: the script itself must start the 2 ranks."""
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    cmd = [sys.executable, os.path.join(ROOT, script), *args]
    return subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=580)


@pytest.mark.timeout(600)
def test_bench_self_launches_n_ranks(tmp_path):
    """The driver's single-process form ``python bench.py --gpus 2`` must run 2 ranks and report them."""
    res = _self_launch(tmp_path, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--ring-mb", "8")
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dist"]["world_size_seen"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["dist"]["engine_collectives"]["all_reduce"] >= 1


def test_bench_world_size_mismatch_exits_nonzero(tmp_path):
    res = _self_launch(tmp_path, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--ring-mb", "8",
                       extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert res.returncode != 0
    assert "disagrees with --gpus" in res.stderr
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]


def _torchrun_json(tmp_path, script, *args):
    res = _self_launch(tmp_path, os.path.join("benchmarks", script), "--gpus", "2", *args)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_fid_two_rank_gloo(tmp_path):
    """BASELINE config #4 at N ranks: sharded updates, one engine all-reduce per state bucket, FID parity."""
    out = _torchrun_json(tmp_path, "bench_fid.py", "--samples", "2000", "--dim", "64", "--batch", "250")
    assert out["n_gpus"] == 2 and out["dist"]["world_size_seen"] == 2 and out["dist"]["backend"] == "gloo"
    assert out["dist"]["engine_collectives"]["all_reduce"] >= 2
    assert out["reference_emulated"]["rel_diff_vs_ours"] < 1e-6
    assert out["rel_diff_fp64_vs_eigh"] < 1e-9


@pytest.mark.timeout(600)
def test_bench_map_two_rank_gloo(tmp_path):
    """BASELINE config #3 at N ranks: list states gathered by the engine, reference per-element sync timed."""
    out = _torchrun_json(tmp_path, "bench_map.py", "--images", "128")
    assert out["n_gpus"] == 2 and out["dist"]["world_size_seen"] == 2
    assert out["dist"]["engine_collectives"]["all_gather"] >= 1
    assert out["reference_sync_s"] is not None and 0 < out["map"] < 1


@pytest.mark.timeout(600)
def test_bench_collection_two_rank_gloo(tmp_path):
    """BASELINE config #5 at N ranks: per-step synced compute of the 20-metric collection against the emulated
    reference collection (parity-checked inside the bench)."""
    out = _torchrun_json(tmp_path, "bench_collection.py", "--steps", "3", "--warmup", "1", "--sync-every-step")
    assert out["n_gpus"] == 2 and out["vs_baseline"] is not None and out["baseline"]["value"] > 0
    assert out["dist"]["world_size_seen"] == 2 and out["dist"]["engine_collectives"]["all_reduce"] >= 1


@pytest.mark.timeout(900)
def test_bench_eight_rank_gloo_rehearsal(tmp_path):
    """8 gloo ranks on the CPU (the driver's N=8 shape, rehearsed without GPUs): bench.py and the config #5 collection
    bench both see world size 8 and report their per-phase split (slowest rank)."""
    res = _self_launch(tmp_path, "bench.py", "--gpus", "8", "--steps", "2", "--warmup", "1", "--ring-mb", "8",
                       "--no-baseline")
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["dist"]["world_size_seen"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["global_batch"] == 8 * 8192 and out["dist"]["engine_collectives"]["all_reduce"] >= 1
    assert set(out["phases_ms_max_over_ranks"]) == {"update_issue_ms", "compute_ms", "closing_sync_ms"}
    coll = _self_launch(tmp_path, os.path.join("benchmarks", "bench_collection.py"), "--gpus", "8", "--steps", "2",
                        "--warmup", "1", "--sync-every-step", "--no-baseline")
    assert coll.returncode == 0, coll.stderr[-3000:]
    c = json.loads([ln for ln in coll.stdout.splitlines() if ln.startswith("{")][0])
    assert c["n_gpus"] == 8 and c["dist"]["world_size_seen"] == 8
    assert set(c["phases_ms_per_step_max_over_ranks"]) == {"update_cls", "update_reg", "compute_cls_incl_sync",
                                                           "compute_reg_incl_sync"}
