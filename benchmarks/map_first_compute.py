"""Config #3: the first compute() of a fresh metric after its 8 updates vs a second compute() of the same states,
per repetition (the first repetition pays the process's one-time costs).  One JSON line per repetition."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_map import make_data  # noqa: E402
from torchmetrics_amd.detection import MeanAveragePrecision  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    preds, target = make_data(512, dev)
    for rep in range(8):
        m = MeanAveragePrecision(class_metrics=True).to(dev)
        torch.cuda.synchronize()
        for i in range(0, 512, 64):
            m.update(preds[i:i + 64], target[i:i + 64])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.compute()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        m._computed = None
        t2 = time.perf_counter()
        m.compute()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        print(json.dumps({"rep": rep, "first_ms": round((t1 - t0) * 1e3, 3), "second_ms": round((t3 - t2) * 1e3, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
