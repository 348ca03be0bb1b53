"""Host-side cost of one ``MulticlassConfusionMatrix.update`` (bench config #2 shapes): wall-clock per call with the
GPU queue kept non-empty, and a cProfile breakdown of where the Python time goes.  Prints JSON + the top entries."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402


def main():
    dev = torch.device("cuda")
    preds = [torch.randn(8192, 1000, device=dev).to(torch.bfloat16) for _ in range(4)]
    target = [torch.randint(0, 1000, (8192,), device=dev) for _ in range(4)]
    m = MulticlassConfusionMatrix(num_classes=1000).to(dev)
    for i in range(50):
        m.update(preds[i % 4], target[i % 4])
    m.compute()
    torch.cuda.synchronize()
    out = {}
    for name, kw in (("validate", {}), ("no_validate", {"validate_args": False})):
        mm = MulticlassConfusionMatrix(num_classes=1000, **kw).to(dev)
        for i in range(20):
            mm.update(preds[i % 4], target[i % 4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(200):
            mm.update(preds[i % 4], target[i % 4])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"host_us": 1e6 * (t1 - t0) / 200, "wall_us": 1e6 * (t2 - t0) / 200}
        t0 = time.perf_counter()
        mm.compute()
        out[name]["compute_us"] = 1e6 * (time.perf_counter() - t0)
    print(json.dumps(out), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(200):
        m.update(preds[i % 4], target[i % 4])
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue())


def compute_costs():
    dev = torch.device("cuda")
    p = torch.randn(8192, 1000, device=dev).to(torch.bfloat16)
    t = torch.randint(0, 1000, (8192,), device=dev)
    res = {}
    for name, kw in (("validate", {}), ("no_validate", {"validate_args": False})):
        mm = MulticlassConfusionMatrix(num_classes=1000, **kw).to(dev)
        times, times_busy = [], []
        for _ in range(60):
            mm.update(p, t)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mm.compute()
            times.append(time.perf_counter() - t0)
            mm.update(p, t)  # compute right behind a queued update (the bench's situation)
            t0 = time.perf_counter()
            mm.compute()
            times_busy.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
        times.sort()
        times_busy.sort()
        res[name] = {"compute_idle_us_median": 1e6 * times[30], "compute_after_update_us_median": 1e6 * times_busy[30]}
    print(json.dumps(res), flush=True)
    mm = MulticlassConfusionMatrix(num_classes=1000).to(dev)
    pr = cProfile.Profile()
    for _ in range(50):
        mm.update(p, t)
        torch.cuda.synchronize()
        pr.enable()
        mm.compute()
        pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(15)
    print(s.getvalue())


if __name__ == "__main__":
    main()
    compute_costs()
