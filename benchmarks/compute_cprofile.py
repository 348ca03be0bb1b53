"""cProfile of a config #5 collection step on the device (host-side cost breakdown): ``--which cls|reg`` (the
classification or the regression collection), ``--update-only`` (no compute)."""
import argparse
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="cls")
    ap.add_argument("--update-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(0)
    if a.which == "cls":
        coll = cls
        x = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
        y = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    else:
        coll = reg
        x = torch.randn(BATCH, generator=g).to(dev)
        y = x + 0.3 * torch.randn(BATCH, generator=g).to(dev)

    def step():
        coll.update(x, y)
        if not a.update_only:
            coll.compute()

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
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
