"""Where config #5's per-step time goes (benchmarks/bench_collection.py --sync-every-step, one GPU): update and
compute of both collections timed separately (host wall-clock, device drained per phase), the fused-compute plan's
members, and a cProfile of the compute calls.  Prints one JSON line; the profile goes to --profile (text)."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--profile", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    cls, reg = build(dev)
    for i in range(10):
        cls.update(logits[i % NBUF], labels[i % NBUF])
        reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()
    torch.cuda.synchronize()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e6

    out = {
        "update_cls_us": timed(lambda i: cls.update(logits[i % NBUF], labels[i % NBUF])),
        "update_reg_us": timed(lambda i: reg.update(xs[i % NBUF], ys[i % NBUF])),
        "compute_cls_us": timed(lambda i: cls.compute()),
        "compute_reg_us": timed(lambda i: reg.compute()),
    }

    def step(i):
        cls.update(logits[i % NBUF], labels[i % NBUF])
        reg.update(xs[i % NBUF], ys[i % NBUF])
        cls.compute(), reg.compute()

    out["step_us"] = timed(step)
    for name, coll in (("cls", cls), ("reg", reg)):
        plan = coll.__dict__.get("_fused_plan")
        out[f"fused_{name}"] = sorted(plan[1].keys) if plan else None
        out[f"fused_rebuilds_{name}"] = coll.__dict__.get("_fused_rebuilds", 0)
    out = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}
    print(json.dumps(out), flush=True)
    if args.profile:
        pr = cProfile.Profile()
        pr.enable()
        for i in range(100):
            step(i)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
        with open(args.profile, "w") as f:
            f.write(s.getvalue())


if __name__ == "__main__":
    main()
