"""cProfile of the config #5 classification collection ``compute()`` on the device (host-side cost breakdown)."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main() -> None:
    dev = torch.device("cuda")
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    labels = torch.randint(0, NC, (BATCH,), generator=g).to(dev)

    def step():
        cls.update(logits, labels)
        cls.compute()

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumtime").print_stats(40)


if __name__ == "__main__":
    main()
