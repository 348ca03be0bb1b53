"""Host cost of one engine sync (``parallel/sync.py sync_state_dicts``) as the world size grows: W gloo ranks on the
CPU sync a config-#5-shaped state set (int64 confusion-matrix / stat-score sums, a float mean, calibration's fp64
bins, Pearson's six ``None``-reduction states through the signed static gather) -- and the same plus a ragged
two-element ``cat`` list, which needs the shape header -- and time it, splitting out the time spent inside the
collectives themselves; ``host_us`` = total - collectives = the engine's own encode / decode work, which must stay flat
in W for config #5 (one all_reduce per bucket, one signed all_gather, no per-rank decode).
Usage: ``python benchmarks/sync_host_scaling.py`` (one process, collectives stubbed: W = 2 ... 64) or
``--gloo`` (spawns W = 2, 4, 8 real gloo ranks on the CPU); one JSON line per W."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from torchmetrics_amd.parallel import sync as eng
    from torchmetrics_amd.utilities.data import dim_zero_cat, dim_zero_mean, dim_zero_sum

    coll = [0.0]
    orig_ag, orig_ar = eng._all_gather_flat, eng._reduce_flat

    def timed_ag(*a, **k):
        t = time.perf_counter()
        try:
            return orig_ag(*a, **k)
        finally:
            coll[0] += time.perf_counter() - t

    def timed_ar(*a, **k):
        t = time.perf_counter()
        try:
            return orig_ar(*a, **k)
        finally:
            coll[0] += time.perf_counter() - t

    eng._all_gather_flat, eng._reduce_flat = timed_ag, timed_ar
    g = torch.Generator().manual_seed(rank)
    states = {"confmat": torch.randint(0, 100, (10, 10)), "tp": torch.randint(0, 100, (10,)),
              "fp": torch.randint(0, 100, (10,)), "mean": torch.randn(5, generator=g),
              "bins": torch.rand(16, 3, dtype=torch.float64, generator=g),
              **{f"p{i}": torch.randn(1, generator=g) for i in range(6)}}
    reds = {"confmat": dim_zero_sum, "tp": dim_zero_sum, "fp": dim_zero_sum, "mean": dim_zero_mean,
            "bins": dim_zero_sum, **{f"p{i}": None for i in range(6)}}
    # config #5's shape: calibration's bins ride as a SUM bucket, Pearson's six states as a signed static gather
    static = {f"p{i}": ((1,), torch.float32, ("Pearson", f"p{i}")) for i in range(6)}
    cat_states = dict(states, preds=[torch.randn(100 + rank, generator=g), torch.randn(7, generator=g)])
    cat_reds = dict(reds, preds=dim_zero_cat)
    out = {"world": world}
    for name, entry in (("config5", (states, reds, static)), ("with_ragged_cat", (cat_states, cat_reds, static))):
        for _ in range(5):
            eng.sync_state_dicts([entry])
        dist.barrier()
        reps = 50
        coll[0] = 0.0
        eng.comm_stats(reset=True)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.sync_state_dicts([entry])
        total = (time.perf_counter() - t0) / reps
        st = eng.comm_stats()
        res = torch.tensor([total, coll[0] / reps], dtype=torch.float64)
        dist.all_reduce(res, op=dist.ReduceOp.MAX)
        out[name] = {"sync_us": round(res[0].item() * 1e6, 1), "collectives_us": round(res[1].item() * 1e6, 1),
                     "host_us": round((res[0].item() - res[1].item()) * 1e6, 1),
                     "meta_all_gather_per_sync": st["meta_all_gather"] / reps}
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def _mock(world: int) -> dict:
    """The engine's own host work at world size W in ONE process: the collectives are replaced by local stand-ins of
    the right shapes (all_reduce: no-op, all_gather: W copies), so nothing but encode / decode is timed -- no gloo
    threads competing with the ranks for the container's CPUs (the --gloo numbers carry that contention)."""
    from torchmetrics_amd.parallel import sync as eng
    from torchmetrics_amd.utilities.data import dim_zero_cat, dim_zero_mean, dim_zero_sum

    saved = (eng._world_size, eng._reduce_flat, eng._all_gather_flat)
    eng._world_size = lambda group: world
    eng._reduce_flat = lambda flat, kind, group, word: None

    def gather(buf, w, group):
        eng._stats["all_gather"] += 1
        return buf.unsqueeze(0).expand(w, -1).contiguous()

    eng._all_gather_flat = gather
    try:
        g = torch.Generator().manual_seed(0)
        states = {"confmat": torch.randint(0, 100, (10, 10)), "tp": torch.randint(0, 100, (10,)),
                  "fp": torch.randint(0, 100, (10,)), "mean": torch.randn(5, generator=g),
                  "bins": torch.rand(16, 3, dtype=torch.float64, generator=g),
                  **{f"p{i}": torch.randn(1, generator=g) for i in range(6)}}
        reds = {"confmat": dim_zero_sum, "tp": dim_zero_sum, "fp": dim_zero_sum, "mean": dim_zero_mean,
                "bins": dim_zero_sum, **{f"p{i}": None for i in range(6)}}
        static = {f"p{i}": ((1,), torch.float32, ("Pearson", f"p{i}")) for i in range(6)}
        cat_states = dict(states, preds=[torch.randn(100, generator=g), torch.randn(7, generator=g)])
        cat_reds = dict(reds, preds=dim_zero_cat)
        out = {"world": world, "mode": "mock"}
        for name, entry in (("config5", (states, reds, static)), ("with_ragged_cat", (cat_states, cat_reds, static))):
            for _ in range(20):
                eng.sync_state_dicts([entry])
            eng.comm_stats(reset=True)
            best = float("inf")
            for _ in range(5):
                t0 = time.perf_counter()
                for _ in range(200):
                    eng.sync_state_dicts([entry])
                best = min(best, (time.perf_counter() - t0) / 200)
            st = eng.comm_stats()
            out[name] = {"host_us": round(best * 1e6, 1), "meta_all_gather_per_sync": st["meta_all_gather"] / 1000}
        return out
    finally:
        eng._world_size, eng._reduce_flat, eng._all_gather_flat = saved


def main() -> None:
    from benchmarks._dist import _free_port

    if "--gloo" not in sys.argv:
        for world in (2, 4, 8, 16, 64):
            print(json.dumps(_mock(world)), flush=True)
        return
    ctx = mp.get_context("spawn")
    for world in (2, 4, 8):
        q = ctx.Queue()
        mp.start_processes(_rank, args=(world, _free_port(), q), nprocs=world, start_method="spawn")
        print(json.dumps(q.get()), flush=True)


if __name__ == "__main__":
    main()
