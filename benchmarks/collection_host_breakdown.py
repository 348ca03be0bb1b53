"""Host-time breakdown of config #5's step (benchmarks/bench_collection.py --sync-every-step) on one GPU: wall-clock
per call of the collection's update / compute pieces, accumulated over the timed steps (the device wait shows up in
``_read_words``, the one status read per compute).  Prints one JSON line of microseconds per step."""
import functools
import json
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402
from torchmetrics_amd import collections as C  # noqa: E402
from torchmetrics_amd.utils import fused_compute as FC  # noqa: E402

ACC = defaultdict(float)


def _timed(owner, name, label):
    fn = getattr(owner, name)

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t0

    setattr(owner, name, w)


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    cls, reg = build(dev)
    MC = C.MetricCollection
    for name in ("update", "_collection_sync", "_defer_device_checks", "_fused_compute", "_finish_device_checks",
                 "_read_words", "_compute_and_reduce"):
        _timed(MC, name, "coll." + name)
    _timed(FC.CollectionPlan, "run", "plan.run")
    _timed(FC.CollectionPlan, "valid", "plan.valid")
    steps = 200
    for i in range(10):
        cls.update(logits[i % NBUF], labels[i % NBUF]), reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()
    torch.cuda.synchronize()
    ACC.clear()
    t0 = time.perf_counter()
    for i in range(steps):
        cls.update(logits[i % NBUF], labels[i % NBUF])
        reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute()
        reg.compute()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    out = {"step_us": round(total / steps * 1e6, 1)}
    out.update({k: round(v / steps * 1e6, 1) for k, v in sorted(ACC.items())})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
