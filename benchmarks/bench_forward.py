"""``metric(preds, target)`` (forward: batch value + accumulation) on ROCm, with forward's in-place SUM merge on and
off (``Metric._inplace_forward_merge``), in one process.  One JSON line per (metric, mode)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402


def run(make, preds, target, inplace, steps=200):
    m = make().cuda()
    m._inplace_forward_merge = inplace
    for i in range(10):
        m(preds[i % len(preds)], target[i % len(target)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        m(preds[i % len(preds)], target[i % len(target)])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6, m.compute()


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    preds = [torch.randn(8192, 1000, device="cuda", generator=g).to(torch.bfloat16) for _ in range(4)]
    target = [torch.randint(0, 1000, (8192,), device="cuda", generator=g) for _ in range(4)]
    cases = {
        "MulticlassConfusionMatrix(1000)": lambda: tm.MulticlassConfusionMatrix(1000),
        "MulticlassAccuracy(1000, macro)": lambda: tm.MulticlassAccuracy(1000),
        "MulticlassF1Score(1000, macro)": lambda: tm.MulticlassF1Score(1000),
    }
    for name, make in cases.items():
        t_off, r_off = run(make, preds, target, False)
        t_on, r_on = run(make, preds, target, True)
        assert torch.equal(r_on, r_off), name
        print(json.dumps({"metric": name, "batch": 8192, "forward_us_out_of_place": round(t_off, 1),
                          "forward_us_in_place": round(t_on, 1), "speedup": round(t_off / t_on, 2)}), flush=True)


if __name__ == "__main__":
    main()
