"""Eager (no GraphedCompute) ``compute()`` cost of the config #5 collections, per member and in total.

Updates the two collections of ``bench_collection.build`` a few times, then times ``cls.compute()`` +
``reg.compute()`` back to back (host loop, then device events), and each member's own ``compute()`` (cache cleared).
Prints one JSON line.  ``--loop N`` only runs N compute pairs (for a rocprofv3 kernel trace).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NC, build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loop", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cls, reg = build(dev)
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16)
    labels = torch.randint(0, NC, (BATCH,), generator=g).to(dev)
    x = torch.randn(BATCH, generator=g).to(dev)
    y = x + 0.3 * torch.randn(BATCH, generator=g).to(dev)
    for _ in range(3):
        cls.update(logits, labels)
        reg.update(x, y)

    def both():
        cls.update(logits, labels)  # invalidates the cached results, as a training step does
        reg.update(x, y)
        cls.compute()
        reg.compute()

    def upd():
        cls.update(logits, labels)
        reg.update(x, y)

    for _ in range(20):
        both()
    torch.cuda.synchronize()
    if args.loop:
        for _ in range(args.loop):
            both()
        torch.cuda.synchronize()
        return
    out = {}
    for name, fn in (("update_pair", upd), ("update_and_compute_pair", both)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            fn()
        torch.cuda.synchronize()
        out[name + "_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
    out["compute_pair_us"] = round(out["update_and_compute_pair_us"] - out["update_pair_us"], 1)
    per = {}
    for coll in (cls, reg):
        for k, m in coll.items(keep_base=True, copy_state=False):
            ts = []
            for _ in range(30):
                m._computed = None
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                m.compute()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e6)
            per[k] = round(sorted(ts)[len(ts) // 2], 1)
    out["per_member_synced_us"] = per
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
