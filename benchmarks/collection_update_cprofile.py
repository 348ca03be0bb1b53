"""cProfile of config #5's steady-state step on ROCm (both collections' update() and compute()): where the host time of
the fused family update, the moments replay and the fused compute goes, builtins included.  Prints the top entries by
internal time."""
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    cls, reg = build(dev)
    for i in range(20):
        cls.update(logits[i % NBUF], labels[i % NBUF]), reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()
    torch.cuda.synchronize()
    steps = 300
    pr = cProfile.Profile()
    pr.enable()
    for i in range(steps):
        cls.update(logits[i % NBUF], labels[i % NBUF])
        reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute()
        reg.compute()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
    print(f"(per step = totals / {steps})")
    print(s.getvalue())


if __name__ == "__main__":
    main()
