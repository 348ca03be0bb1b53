"""The emulated reference of BASELINE config #2 on its own (for a kernel trace that contains only the baseline's
kernels): the same 406 MB ring, W warm-up updates and K timed updates + compute as bench.py."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import BATCH, DEFAULT_RING_MB, NUM_CLASSES, _data  # noqa: E402
from benchmarks.reference_path import ReferenceEmulatedConfusionMatrix  # noqa: E402


def main(steps: int = 200, warmup: int = 20) -> None:
    dev = torch.device("cuda")
    preds, target = _data(dev, 0, DEFAULT_RING_MB)
    ref = ReferenceEmulatedConfusionMatrix(NUM_CLASSES, dev)
    for i in range(warmup):
        ref.update(preds[i % len(preds)], target[i % len(preds)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ref.update(preds[(warmup + i) % len(preds)], target[(warmup + i) % len(preds)])
    ref.compute()
    torch.cuda.synchronize()
    print(f"reference emulation: {steps / (time.perf_counter() - t0):.1f} updates/s (batch {BATCH})")


if __name__ == "__main__":
    main()
