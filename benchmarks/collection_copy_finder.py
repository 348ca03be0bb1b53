"""Which ATen ops of config #5's steady-state step issue device copies (torch.profiler, Python stacks): prints the copy
ops with their call sites, one JSON line per distinct site."""
import json
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    cls, reg = build(dev)
    for i in range(10):
        cls.update(logits[i % NBUF], labels[i % NBUF]), reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()
    torch.cuda.synchronize()
    sites = Counter()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
        for i in range(20):
            cls.update(logits[i % NBUF], labels[i % NBUF]), reg.update(xs[i % NBUF], ys[i % NBUF])
            cls.compute(), reg.compute()
        torch.cuda.synchronize()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::_to_copy", "aten::clone", "aten::item", "aten::_local_scalar_dense",
                       "aten::cat", "aten::index", "aten::nonzero"):
            stack = [f for f in (ev.stack or []) if "torchmetrics_amd" in f or "benchmarks" in f][:4]
            sites[(ev.name, " <- ".join(stack))] += 1
    for (name, stack), n in sites.most_common():
        print(json.dumps({"op": name, "per_step": n / 20, "site": stack}), flush=True)


if __name__ == "__main__":
    main()
