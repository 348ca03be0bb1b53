"""Where the fixed cost of bench.py's short timed region goes (20 updates + compute, config #2 shapes): host
timestamps around the launches / compute / final sync and device events around the update kernels."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchmetrics_amd.classification import MulticlassConfusionMatrix  # noqa: E402


def main():
    dev = torch.device("cuda")
    k = 26
    g = torch.Generator(device=dev).manual_seed(0)
    preds = [torch.randn(8192, 1000, device=dev, generator=g).to(torch.bfloat16) for _ in range(k)]
    target = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(k)]
    m = MulticlassConfusionMatrix(num_classes=1000).to(dev)
    rows = []
    for rep in range(6):
        for i in range(5):
            m.update(preds[i], target[i])
        m.compute()
        m.reset()
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0 = time.perf_counter()
        e0.record()
        for i in range(20):
            m.update(preds[(5 + i) % k], target[(5 + i) % k])
        e1.record()
        t1 = time.perf_counter()
        m.compute()
        t2 = time.perf_counter()
        e2.record()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append({"launch_us": 1e6 * (t1 - t0), "compute_us": 1e6 * (t2 - t1), "sync_us": 1e6 * (t3 - t2),
                     "total_us": 1e6 * (t3 - t0), "dev_updates_us": 1e3 * e0.elapsed_time(e1),
                     "dev_compute_us": 1e3 * e1.elapsed_time(e2)})
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
