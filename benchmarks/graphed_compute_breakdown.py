"""Per-phase host / device time of ``GraphedCompute`` on the config #5 collections (bench_collection.py's metrics)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402
from torchmetrics_amd.utils.graphs import GraphedCompute  # noqa: E402


def timed(fn, reps=200, sync=True):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    host = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e6
    return round(host, 1), round(wall, 1)


def main():
    dev = torch.device("cuda", 0)
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(0)
    lg = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    lb = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    x = torch.randn(BATCH, generator=g).to(dev)
    y = x + 0.3 * torch.randn(BATCH, generator=g).to(dev)
    for _ in range(3):
        cls.update(lg, lb)
        reg.update(x, y)
    gc, gr = GraphedCompute(cls), GraphedCompute(reg)
    out = {"eager_members_cls": [n for n, _ in gc._eager], "eager_members_reg": [n for n, _ in gr._eager],
           "reasons": {**gc._capture_errors, **gr._capture_errors}}
    gb = GraphedCompute(cls, reg)
    out["graphed_both_call_us"] = timed(gb)
    out["graphed_cls_call_us"] = timed(gc)
    out["graphed_reg_call_us"] = timed(gr)
    out["replay_only_cls_us"] = timed(gc._graph.replay)
    out["replay_only_reg_us"] = timed(gr._graph.replay)
    # device time of one replay
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, gg in (("cls", gc), ("reg", gr)):
        ts = []
        for _ in range(20):
            e0.record()
            gg._graph.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out[f"replay_device_{name}_us"] = round(sorted(ts)[10], 1)
    out["replay_and_errsync_cls_us"] = timed(lambda: gc._replay())
    out["replay_sections_cls_us"] = replay_sections(gc)
    out["eager_cls_compute_us"] = timed(lambda: ([setattr(m, "_computed", None) for m in cls.values(copy_state=False)],
                                                 cls.compute()))
    ece = cls["ece"]

    def ece_compute():
        ece._computed = None
        ece.compute()

    out["ece_compute_us"] = timed(ece_compute)
    t = torch.zeros(1, dtype=torch.int32, device=dev)
    out["item_sync_us"] = timed(lambda: t.item())
    pinned = torch.zeros(1, dtype=torch.int32, pin_memory=True)

    def pinned_read():
        pinned.copy_(t, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return int(pinned[0])

    out["pinned_sync_us"] = timed(pinned_read)
    out["empty_sync_us"] = timed(lambda: torch.cuda.current_stream().synchronize())
    print(json.dumps(out), flush=True)




def replay_sections(gc, reps=200):
    """Host time of each section of GraphedCompute._replay (same steps, timed)."""
    import collections

    acc = collections.defaultdict(float)
    for _ in range(reps):
        t = time.perf_counter()
        gc._graph.replay()
        t1 = time.perf_counter(); acc["replay"] += t1 - t; t = t1
        from torchmetrics_amd.utils.graphs import _contig_strides
        copies = {dt: buf.clone() for dt, buf in gc._outs.items()}
        leaves = [None] * gc._n_leaves
        for i, dt, shape, off in gc._leaf_views:
            leaves[i] = torch.as_strided(copies[dt], shape, _contig_strides(shape), off)
        t1 = time.perf_counter(); acc["copy_out"] += t1 - t; t = t1
        torch.cuda.current_stream().synchronize()
        t1 = time.perf_counter(); acc["sync"] += t1 - t; t = t1
        codes = gc._host_words.tolist()
        any(codes)
        t1 = time.perf_counter(); acc["words"] += t1 - t; t = t1
        from torchmetrics_amd.utils.graphs import _rebuild
        {n: _rebuild(spec, leaves) for (n, _), spec in zip(gc._graphed, gc._spec)}
        t1 = time.perf_counter(); acc["rebuild"] += t1 - t; t = t1
    return {k: round(v / reps * 1e6, 1) for k, v in acc.items()}


if __name__ == "__main__":
    main()
