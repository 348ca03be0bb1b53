"""List every device->host synchronisation triggered by a metric step (``torch.cuda.set_sync_debug_mode``).

Runs a few steps of the config #5 collection (benchmarks/bench_collection.py) with sync debugging set to "warn" and
prints each distinct synchronising call site (innermost torchmetrics_amd frame) with its count.
"""
import collections
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main() -> None:
    dev = torch.device("cuda")
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    labels = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    x = torch.randn(BATCH, generator=g).to(dev)
    y = x + 0.1
    for _ in range(3):  # warm up (first update decides compute groups)
        cls.update(logits, labels)
        reg.update(x, y)
    torch.cuda.synchronize()
    sites = collections.Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        frames = [f for f in traceback.extract_stack() if "torchmetrics_amd" in f.filename]
        where = f"{frames[-1].filename.split('torchmetrics_amd/')[-1]}:{frames[-1].lineno} {frames[-1].line}" if frames else "?"
        sites[where] += 1

    warnings.showwarning = hook
    torch.cuda.set_sync_debug_mode("warn")
    for _ in range(5):
        cls.update(logits, labels)
        reg.update(x, y)
    torch.cuda.set_sync_debug_mode("default")
    print(f"update-path syncs over 5 steps: {sum(sites.values())}")
    for k, v in sites.most_common():
        print(f"  {v:4d}  {k}")
    sites.clear()
    torch.cuda.set_sync_debug_mode("warn")
    cls.compute()
    reg.compute()
    torch.cuda.set_sync_debug_mode("default")
    print(f"compute-path syncs: {sum(sites.values())}")
    for k, v in sites.most_common(15):
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
