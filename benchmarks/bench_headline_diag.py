"""Where the headline's short-run time goes.

For the bench.py config (MulticlassConfusionMatrix(1000), 8192 x 1000 bf16) measure, on one GPU:

* ``steady_us``: per-update wall time over 500 updates (GPU-bound steady state);
* ``short_region_ms``: the driver's region (20 updates + compute, barrier/synchronize bracketed);
* ``updates_only_ms`` (20 updates + synchronize) and ``compute_only_us`` (a compute after a fresh update);
* ``host_update_us``: host time of one update() call (no synchronize);
* the same with the input ring larger than the 256 MB MALL (``ring_mb``), i.e. logits streamed from HBM, and the
  resulting effective HBM bandwidth of the argmax+histogram kernel.

Usage: python benchmarks/bench_headline_diag.py [--rings 64,400]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402

C, N = 1000, 8192


def make_ring(ring_mb: int, dev):
    per = N * C * 2
    k = max(2, (ring_mb * 2**20 + per - 1) // per)
    g = torch.Generator(device=dev).manual_seed(0)
    preds = [torch.randn(N, C, generator=g, device=dev).to(torch.bfloat16) for _ in range(k)]
    target = [torch.randint(0, C, (N,), generator=g, device=dev) for _ in range(k)]
    return preds, target


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rings", default="64,400")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for ring_mb in [int(x) for x in args.rings.split(",")]:
        preds, target = make_ring(ring_mb, dev)
        k = len(preds)
        m = MulticlassConfusionMatrix(num_classes=C).to(dev)
        for i in range(20):
            m.update(preds[i % k], target[i % k])
        m.compute()
        m.reset()
        torch.cuda.synchronize()
        # steady state
        t0 = time.perf_counter()
        for i in range(500):
            m.update(preds[i % k], target[i % k])
        torch.cuda.synchronize()
        steady = (time.perf_counter() - t0) / 500 * 1e6
        # host cost of update() alone
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(50):
            m.update(preds[i % k], target[i % k])
        host = (time.perf_counter() - t0) / 50 * 1e6
        torch.cuda.synchronize()
        # driver's short region, repeated
        shorts, upd_only, comp = [], [], []
        for rep in range(10):
            m.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(20):
                m.update(preds[(i + rep) % k], target[(i + rep) % k])
            m.compute()
            torch.cuda.synchronize()
            shorts.append((time.perf_counter() - t0) * 1e3)
            m.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(20):
                m.update(preds[(i + rep) % k], target[(i + rep) % k])
            torch.cuda.synchronize()
            upd_only.append((time.perf_counter() - t0) * 1e3)
            m.update(preds[0], target[0])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m.compute()
            torch.cuda.synchronize()
            comp.append((time.perf_counter() - t0) * 1e6)
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        print(json.dumps({
            "ring_mb": round(k * N * C * 2 / 2**20, 1), "buffers": k, "steady_us": round(steady, 2),
            "updates_per_s_steady": round(1e6 / steady, 1), "host_update_us": round(host, 2),
            "short_region_ms": round(med(shorts), 4), "short_updates_per_s": round(20 / med(shorts) * 1e3, 1),
            "updates_only_ms": round(med(upd_only), 4), "compute_only_us": round(med(comp), 2),
            "eff_TBps_steady": round(N * C * 2 / (steady * 1e-6) / 1e12, 2),
        }), flush=True)
        del preds, target
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
