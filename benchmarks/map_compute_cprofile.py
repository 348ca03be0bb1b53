"""cProfile of config #3's ``MeanAveragePrecision.compute()`` on the device (host-side op costs)."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_map import make_data  # noqa: E402
from torchmetrics_amd.detection import MeanAveragePrecision  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    preds, target = make_data(512, dev)
    m = MeanAveragePrecision(class_metrics=True, extended_summary="--extended" in sys.argv).to(dev)
    for i in range(0, 512, 64):
        m.update(preds[i:i + 64], target[i:i + 64])
    for _ in range(2):
        m._computed = None
        m.compute()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        m._computed = None
        m.compute()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(45)


if __name__ == "__main__":
    main()
