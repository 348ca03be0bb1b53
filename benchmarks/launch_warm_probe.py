"""Is the headline's slow first timed region a lazily-initialised HIP launch path?  One fresh process per run:
``--prelaunch N`` issues N one-element ``add_`` kernels (and synchronises) before the usual W warm-up updates, then
the bench's exact timed region (20 updates + compute, barrier + synchronize on both sides) runs once.  Prints one
JSON line: the region in us and the per-update host times inside it."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prelaunch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    preds, target = bench._data(dev, 0, bench.DEFAULT_RING_MB)
    m = MulticlassConfusionMatrix(num_classes=bench.NUM_CLASSES).to(dev)
    if args.prelaunch:
        x = torch.zeros(1, device=dev)
        for _ in range(args.prelaunch):
            x.add_(1)
        torch.cuda.synchronize()
    bench._warm(m, preds, target, args.warmup)
    nbuf = len(preds)
    torch.cuda.synchronize()
    per = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        a = time.perf_counter()
        m.update(preds[(args.warmup + i) % nbuf], target[(args.warmup + i) % nbuf])
        per.append(round((time.perf_counter() - a) * 1e6, 1))
    t1 = time.perf_counter()
    m.compute()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"prelaunch": args.prelaunch, "region_us": round((t2 - t0) * 1e6, 1),
                      "launch_phase_us": round((t1 - t0) * 1e6, 1), "per_update_us": per}), flush=True)


if __name__ == "__main__":
    main()
