"""Host-time detail of config #5's step pieces on one GPU, each timed with the device idle before it (so a piece's
wall time is its own host work plus its own kernels' latency, not the queue it waits behind): the two collections'
update() and compute(), and inside compute() the collection's phases and each member's own compute().  Prints one
JSON line of microseconds per step (median over the timed steps)."""
import functools
import json
import os
import statistics
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402
from torchmetrics_amd import collections as C  # noqa: E402
from torchmetrics_amd.utils import fused_compute as FC  # noqa: E402
from torchmetrics_amd.utils import fused_update as FU  # noqa: E402

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
    for name in ("_collection_sync", "_defer_device_checks", "_fused_compute", "_finish_device_checks", "_read_words",
                 "_fused_update", "_replay_moments", "_compute_groups_create_state_ref"):
        _timed(MC, name, "coll." + name)
    _timed(FC.CollectionPlan, "run", "fused_compute.run")
    _timed(FC.CollectionPlan, "valid", "fused_compute.valid")
    _timed(FU.FamilyPlan, "run", "family.run")
    for coll, tag in ((cls, "cls"), (reg, "reg")):
        for n, m in coll.items(keep_base=True, copy_state=False):
            fn = m.__dict__.get("compute")
            if fn is not None:
                _timed(m, "compute", f"member.{tag}.{n}.compute")
    steps = 200
    for i in range(10):
        cls.update(logits[i % NBUF], labels[i % NBUF]), reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()
    torch.cuda.synchronize()
    pieces = defaultdict(list)
    acc_steps = []
    for i in range(steps):
        ACC.clear()
        for label, fn in (("update_cls", lambda: cls.update(logits[i % NBUF], labels[i % NBUF])),
                          ("update_reg", lambda: reg.update(xs[i % NBUF], ys[i % NBUF])),
                          ("compute_cls", cls.compute), ("compute_reg", reg.compute)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            pieces[label].append(time.perf_counter() - t0)
        acc_steps.append(dict(ACC))
    torch.cuda.synchronize()
    out = {k: round(statistics.median(v) * 1e6, 1) for k, v in pieces.items()}
    keys = sorted({k for a in acc_steps for k in a})
    out["detail"] = {k: round(statistics.median([a.get(k, 0.0) for a in acc_steps]) * 1e6, 1) for k in keys}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
