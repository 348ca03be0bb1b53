#!/usr/bin/env python3
"""Headline benchmark: ``MulticlassConfusionMatrix(num_classes=1000)`` on batches of 8192 bf16 logits, DDP sync.

BASELINE.json config #2 ("MulticlassConfusionMatrix num_classes=1000, batch=8192 bf16, DDP sync over N x MI355X").
Metric: metric-updates/sec summed over the node (each rank updates its own metric on its own 8192-row batches;
weak scaling: per-GPU work is fixed).  The timed region of one run is K ``update`` calls followed by one synced
``compute()`` (RCCL all-reduce of the 1000x1000 int64 state), bracketed by barrier + ``torch.cuda.synchronize()``;
the max over ranks is reported.  ``compute_ms`` (sync + compute wall-clock) is measured separately.

The same loop is also run through an op-for-op emulation of the reference implementation (``benchmarks/reference_path.py``)
on the same data in the same process; ``vs_baseline`` = ours / emulated reference.

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``.  ``--gpus N`` always means N ranks: under a launcher
(``torch.distributed.run``, ``WORLD_SIZE`` set) the world size must equal N or the run exits non-zero; without one,
N > 1 spawns ``torch.distributed.run --nproc-per-node N`` itself as a child process before any GPU call
(``benchmarks/_dist.py`` ``launch``).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

NUM_CLASSES = 1000
BATCH = 8192
# input ring: 400 MB by default, larger than MI355X's 256 MB MALL (Infinity Cache), so every update streams its
# logits from HBM as it would straight after a model forward on another batch (--ring-mb 64 = cache-resident ring)
DEFAULT_RING_MB = 400


def _setup(gpus: int):
    from benchmarks._dist import launch

    launch(gpus, __file__)  # returns only inside one of the ``gpus`` ranks
    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == gpus, (world, gpus)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1:
        backend = "nccl" if device.type == "cuda" else "gloo"
        dist.init_process_group(backend, rank=rank, world_size=world)
    return world, rank, device


def _barrier_sync(device: torch.device, world: int) -> None:
    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()


def _max_over_ranks(x: float, device: torch.device, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _data(device: torch.device, rank: int, ring_mb: int):
    """The input ring as ONE [k, 8192, 1000] bf16 allocation (plus one [k, 8192] int64 target block), filled in
    place: a single large segment instead of k separate ones (measured: the first timed region after k separate
    allocations ran ~25 % slower, profiles/r03_first_region.md)."""
    per = BATCH * NUM_CLASSES * 2
    k = max(2, (ring_mb * 2**20 + per - 1) // per)
    gdev = device if device.type == "cuda" else torch.device("cpu")
    g = torch.Generator(device=gdev).manual_seed(1234 + rank)
    ring = torch.empty(k, BATCH, NUM_CLASSES, dtype=torch.bfloat16, device=gdev)
    for i in range(k):
        ring[i].copy_(torch.randn(BATCH, NUM_CLASSES, generator=g, device=gdev))
    target = torch.randint(0, NUM_CLASSES, (k, BATCH), generator=g, device=gdev)
    return list(ring.unbind(0)), list(target.unbind(0))


def _warm(metric, preds, target, warmup: int) -> None:
    """W untimed warm-up updates, then compute() and reset() (the state the timed region starts from)."""
    nbuf = len(preds)
    for i in range(warmup):
        metric.update(preds[i % nbuf], target[i % nbuf])
    metric.compute()
    _reset(metric)


def _timed(metric, preds, target, steps: int, warmup: int, device, world):
    """EXACTLY ``steps`` updates and one synced compute(), bracketed by barrier + synchronize; then the synced
    compute() wall-clock on its own (5 reps)."""
    nbuf = len(preds)
    _barrier_sync(device, world)
    t0 = time.perf_counter()
    for i in range(steps):
        metric.update(preds[(warmup + i) % nbuf], target[(warmup + i) % nbuf])
    t1 = time.perf_counter()
    result = metric.compute()
    t2 = time.perf_counter()
    _barrier_sync(device, world)
    t3 = time.perf_counter()
    elapsed = t3 - t0
    # host-side phases of the timed region: issuing the K updates, compute() (sync + validation read: it waits for the
    # device to drain), the closing barrier + synchronize
    phases = {"update_issue_ms": (t1 - t0) * 1e3, "compute_ms": (t2 - t1) * 1e3, "closing_sync_ms": (t3 - t2) * 1e3}
    # separate measurement of the synced compute wall-clock
    _barrier_sync(device, world)
    c0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        if hasattr(metric, "_computed"):
            metric._computed = None
        result = metric.compute()
    _barrier_sync(device, world)
    compute_ms = (time.perf_counter() - c0) / reps * 1e3
    return elapsed, compute_ms, result, phases


def _reset(metric) -> None:
    if hasattr(metric, "reset"):
        metric.reset()
    else:
        metric.confmat.zero_()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-baseline", action="store_true", help="skip the in-run reference-emulation baseline")
    ap.add_argument("--ring-mb", type=int, default=DEFAULT_RING_MB, help="size of the input ring (MB)")
    args = ap.parse_args()

    world, rank, device = _setup(args.gpus or int(os.environ.get("WORLD_SIZE", "1")))
    from torchmetrics_amd.classification import MulticlassConfusionMatrix

    preds, target = _data(device, rank, args.ring_mb)
    from torchmetrics_amd.parallel.sync import comm_stats

    comm_stats(reset=True)

    ours = MulticlassConfusionMatrix(num_classes=NUM_CLASSES).to(device)
    ref = None
    if not args.no_baseline:
        from benchmarks.reference_path import ReferenceEmulatedConfusionMatrix

        ref = ReferenceEmulatedConfusionMatrix(NUM_CLASSES, device)
    _warm(ours, preds, target, args.warmup)
    t_ours, cms_ours, res_ours, phases = _timed(ours, preds, target, args.steps, args.warmup, device, world)
    comms = comm_stats()
    t_ours = _max_over_ranks(t_ours, device, world)
    cms_ours = _max_over_ranks(cms_ours, device, world)
    phases = {k: round(_max_over_ranks(v, device, world), 4) for k, v in phases.items()}  # slowest rank per phase

    base_val = None
    t_ref = cms_ref = None
    if ref is not None:
        _warm(ref, preds, target, args.warmup)
        t_ref, cms_ref, res_ref, _ = _timed(ref, preds, target, args.steps, args.warmup, device, world)
        t_ref = _max_over_ranks(t_ref, device, world)
        cms_ref = _max_over_ranks(cms_ref, device, world)
        if not torch.equal(res_ref.to(res_ours.device), res_ours):
            raise RuntimeError("benchmark parity failure: confusion matrices differ from the reference emulation")
        base_val = world * args.steps / t_ref

    value = world * args.steps / t_ours
    if rank == 0:
        out = {
            "metric": "metric-updates/sec (whole node)",
            "value": round(value, 2),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_ours / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / base_val, 3) if base_val else None,
            "dtype": "bf16",
            "data": "synthetic (randn bf16 logits, uniform int64 targets; fixed seeds; HBM-streamed input ring)",
            "config": {
                "model": "MulticlassConfusionMatrix(num_classes=1000)",
                "global_batch": BATCH * world,
                "seq_len": 1,
                "parallelism": f"dp{world}",
            },
            "compute_ms": round(cms_ours, 4),
            "phases_ms_max_over_ranks": phases,
            "input_ring_mb": round(len(preds) * BATCH * NUM_CLASSES * 2 / 2**20, 1),
            "dist": {
                "world_size_seen": dist.get_world_size() if world > 1 else 1,
                "backend": dist.get_backend() if world > 1 else None,
                "engine_collectives": comms,
            },
            "samples_per_s": round(value * BATCH, 1),
            "baseline": {
                "impl": "emulated reference op chain: torchmetrics 1.4.0dev op sequence re-run in this process (benchmarks/reference_path.py; the reference package is not importable on the box)",
                "value": round(base_val, 2) if base_val else None,
                "ms_per_step": round(t_ref / args.steps * 1e3, 4) if t_ref else None,
                "compute_ms": round(cms_ref, 4) if cms_ref else None,
            },
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
