"""cProfile of MeanAveragePrecision.update on the bench_map batches (512 images, 64 per call) on ROCm."""
import cProfile
import io
import pstats
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_map import BATCH, make_data  # noqa: E402
from torchmetrics_amd.detection import MeanAveragePrecision  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    preds, target = make_data(512, dev)
    for _ in range(3):
        m = MeanAveragePrecision(class_metrics=True).to(dev)
        for i in range(0, 512, BATCH):
            m.update(preds[i:i + BATCH], target[i:i + BATCH])
    torch.cuda.synchronize()
    m = MeanAveragePrecision(class_metrics=True).to(dev)
    t0 = time.perf_counter()
    for i in range(0, 512, BATCH):
        m.update(preds[i:i + BATCH], target[i:i + BATCH])
    torch.cuda.synchronize()
    print("update_s", time.perf_counter() - t0)
    m = MeanAveragePrecision(class_metrics=True).to(dev)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(0, 512, BATCH):
        m.update(preds[i:i + BATCH], target[i:i + BATCH])
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(20)
    print(s.getvalue())


if __name__ == "__main__":
    main()
