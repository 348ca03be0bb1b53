"""Why bench.py's single 20-step region (after only 5 warm-up updates) runs slower than later regions: per-update host
timestamps and device events, for the region exactly as bench.py runs it and for variants
(a) repeated regions, (b) the ring's buffers read once by a trivial kernel beforehand (TLB / cache warm),
(c) a 2 ms device-busy period right before the region (clock ramp)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402

C, B, K = 1000, 8192, 26


def region_noevents(m, preds, target, start, steps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m.update(preds[(start + i) % K], target[(start + i) % K])
    t1 = time.perf_counter()
    m.compute()
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    return {"noevents_total_us": round(1e6 * (t3 - t0), 1), "launch_us": round(1e6 * (t1 - t0), 1),
            "compute_us": round(1e6 * (t2 - t1), 1), "sync_us": round(1e6 * (t3 - t2), 1)}


def region(m, preds, target, start, steps=20):
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ts = []
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        m.update(preds[(start + i) % K], target[(start + i) % K])
        ts.append(time.perf_counter())
    ev[1].record()
    m.compute()
    t_c = time.perf_counter()
    ev[2].record()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    per = [1e6 * (b - a) for a, b in zip([t0] + ts[:-1], ts)]
    return {"total_us": round(1e6 * (t_end - t0), 1), "launch_us": round(1e6 * (ts[-1] - t0), 1),
            "first3_us": [round(x, 1) for x in per[:3]], "median_us": round(sorted(per)[len(per) // 2], 2),
            "compute_us": round(1e6 * (t_c - ts[-1]), 1), "sync_us": round(1e6 * (t_end - t_c), 1),
            "dev_updates_us": round(1e3 * ev[0].elapsed_time(ev[1]), 1),
            "dev_compute_us": round(1e3 * ev[1].elapsed_time(ev[2]), 1)}


def fresh(variant):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1234)
    preds = [torch.randn(B, C, generator=g, device=dev).to(torch.bfloat16) for _ in range(K)]
    target = [torch.randint(0, C, (B,), generator=g, device=dev) for _ in range(K)]
    m = MulticlassConfusionMatrix(num_classes=C).to(dev)
    if variant == "touch_ring":
        s = torch.zeros((), device=dev)
        for p in preds:
            s += p[:, 0].float().sum()
        torch.cuda.synchronize()
    for i in range(5):
        m.update(preds[i], target[i])
    m.compute()
    if variant == "inplace_reset":
        m.confmat.zero_()  # keep the state block the warm-up updates touched
        m._update_count = 0
    else:
        m.reset()
    if variant == "busy_2ms":
        x = torch.randn(4096, 4096, device=dev)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.002:
            x = x * 1.0000001
    torch.cuda.synchronize()
    if variant == "noevents":
        out = [region_noevents(m, preds, target, 5)]
        for r in range(2):
            m.reset()
            out.append(region_noevents(m, preds, target, 5 + 20 * (r + 1)))
        return out
    out = [region(m, preds, target, 5)]
    if variant == "plain":
        for r in range(3):
            m.reset()
            out.append(region(m, preds, target, 5 + 20 * (r + 1)))
    return out


def main():
    res = {}
    for v in ("plain", "inplace_reset", "plain", "inplace_reset", "noevents"):
        res.setdefault(v, []).append(fresh(v))
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
