"""Host and device time of each phase of the graphed config #5 step (bench_collection.py --graph --sync-every-step).

Phases: the grouped update replay, the eager calibration update, the GraphedCompute call.  Device times come from
events around each phase on an otherwise idle stream (synchronised between phases); host times from the
un-synchronised loop.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, NBUF, build  # noqa: E402
from torchmetrics_amd import MetricCollection  # noqa: E402
from torchmetrics_amd.utils.graphs import GraphedCompute, GraphedUpdate, UpdateGroup  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    ece = cls["ece"]
    cls_graph = MetricCollection({k: m for k, m in cls.items(keep_base=True) if k != "ece"}, compute_groups=True)
    group = UpdateGroup((cls_graph, 2), (reg, 2))
    gu = [GraphedUpdate(group, logits[i], labels[i], xs[i], ys[i], bind_inputs=True) for i in range(NBUF)]
    for i in range(2):
        gu[i]()
        ece.update(logits[i], labels[i])
    gc = GraphedCompute(cls, reg)
    phases = {"update_replay": lambda i: gu[i % NBUF](), "ece_update": lambda i: ece.update(logits[i % NBUF],
                                                                                                labels[i % NBUF]),
              "compute": lambda i: gc()}
    out = {}
    for name, fn in phases.items():
        for i in range(20):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dev_t, host_t = [], []
        for i in range(100):
            torch.cuda.synchronize()
            e0.record()
            t0 = time.perf_counter()
            fn(i)
            host_t.append((time.perf_counter() - t0) * 1e6)
            e1.record()
            e1.synchronize()
            dev_t.append(e0.elapsed_time(e1) * 1e3)
        med = lambda v: round(sorted(v)[len(v) // 2], 1)  # noqa: E731
        out[name] = {"host_us": med(host_t), "device_us": med(dev_t)}
    # throughput of back-to-back loops (no sync inside unless the phase syncs itself)
    loops = {
        "loop_update_only": lambda i: gu[i % NBUF](),
        "loop_update_ece": lambda i: (gu[i % NBUF](), ece.update(logits[i % NBUF], labels[i % NBUF])),
        "loop_compute_only": lambda i: gc(),
        "step_us": lambda i: (gu[i % NBUF](), ece.update(logits[i % NBUF], labels[i % NBUF]), gc()),
    }
    for name, fn in loops.items():
        for i in range(10):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(300):
            fn(i)
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t0) / 300 * 1e6, 1)
    out["update_graph_nodes"] = gu[0].graph.__class__.__name__
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
