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
    ap.add_argument("--cprofile", action="store_true")
    ap.add_argument("--phases", action="store_true")
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
    if args.phases:
        from torchmetrics_amd.collections import MetricCollection

        acc = {}

        def timed(name, fn):
            def w(*a, **k):
                t0 = time.perf_counter()
                try:
                    return fn(*a, **k)
                finally:
                    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return w

        for name in ("_collection_sync", "_defer_device_checks", "_finish_device_checks", "_read_words", "items",
                     "_compute_and_reduce"):
            setattr(MetricCollection, name, timed(name, getattr(MetricCollection, name)))
        members = [m for c in (cls, reg) for m in c.values(copy_state=False)]
        for m in members:
            type(m).compute.__wrapped__ if False else None
        for _ in range(200):
            both()
        torch.cuda.synchronize()
        print(json.dumps({k: round(v / 200 * 1e6, 1) for k, v in acc.items()}), flush=True)
        return
    if args.cprofile:
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        for _ in range(200):
            both()
        torch.cuda.synchronize()
        pr.disable()
        st = pstats.Stats(pr)
        st.sort_stats("cumtime").print_stats(45)
        st.sort_stats("tottime").print_stats(30)
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
    # compute() alone on unchanged states (results un-cached, device idle): the host cost of the eager path
    for name, coll in (("cls", cls), ("reg", reg)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            for m in coll.values(copy_state=False):
                m._computed = None
            coll.compute()
        torch.cuda.synchronize()
        out[f"{name}_compute_idle_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 1)
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
    from torchmetrics_amd.utils.deferred import suppress

    for label, ctx in (("per_member_host_us", None), ("per_member_host_nochecks_us", suppress)):
        per = {}
        for coll in (cls, reg):
            for k, m in coll.items(keep_base=True, copy_state=False):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(100):
                    m._computed = None
                    if ctx is None:
                        m.compute()
                    else:
                        with ctx():
                            m.compute()
                per[k] = round((time.perf_counter() - t0) / 100 * 1e6, 1)
                torch.cuda.synchronize()
        out[label] = per
        out[label.replace("per_member", "sum")] = round(sum(per.values()), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
