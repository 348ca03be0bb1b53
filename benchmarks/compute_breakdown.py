"""Per-metric ``compute()`` wall-clock of the config #5 collection members after K updates (GPU)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main(steps: int = 50) -> None:
    dev = torch.device("cuda")
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    labels = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    x = torch.randn(BATCH, generator=g).to(dev)
    y = x + 0.1
    for _ in range(steps):
        cls.update(logits, labels)
        reg.update(x, y)
    torch.cuda.synchronize()
    for col in (cls, reg):
        for name, m in col.items(keep_base=True, copy_state=False):
            for rep in range(3):
                m._computed = None
                torch.cuda.synchronize()
                t = time.perf_counter()
                m.compute()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) * 1e3
            print(f"{name:10s} {dt:8.3f} ms")
    for col in (cls, reg):
        for _, m in col.items(keep_base=True, copy_state=False):
            m._computed = None
        torch.cuda.synchronize()
        t = time.perf_counter()
        col.compute()
        torch.cuda.synchronize()
        print(f"collection compute {(time.perf_counter() - t) * 1e3:8.3f} ms")


if __name__ == "__main__":
    main()
