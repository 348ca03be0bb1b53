"""Per-member cost of the config #5 collection: each metric updated alone (us per update, device-synchronised),
then each compute group as the collection runs it.  Prints one JSON line per entry."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmarks.bench_collection import BATCH, NBUF, NC, build  # noqa: E402


def timed(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    h = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    return (h - t0) / n * 1e6, (t1 - t0) / n * 1e6


def main():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(7)
    logits = [torch.randn(BATCH, NC, generator=g).to(dev, torch.bfloat16) for _ in range(NBUF)]
    labels = [torch.randint(0, NC, (BATCH,), generator=g).to(dev) for _ in range(NBUF)]
    xs = [torch.randn(BATCH, generator=g).to(dev) for _ in range(NBUF)]
    ys = [(x + 0.3 * torch.randn(BATCH, generator=g).to(dev)) for x in xs]
    cls, reg = build(dev)
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % NBUF
        return it[0]

    for name, m in list(cls.items(keep_base=True)) + list(reg.items(keep_base=True)):
        m = m.clone()
        is_reg = name in reg.keys(keep_base=True)
        def f(m=m, is_reg=is_reg):
            i = nxt()
            if is_reg:
                m.update(xs[i], ys[i])
            else:
                m.update(logits[i], labels[i])
        host, total = timed(f)
        print(json.dumps({"metric": name, "host_us": round(host, 1), "total_us": round(total, 1)}), flush=True)
    def fc():
        i = nxt()
        cls.update(logits[i], labels[i])
    def fr():
        i = nxt()
        reg.update(xs[i], ys[i])
    for nm, f in (("collection_cls", fc), ("collection_reg", fr)):
        host, total = timed(f)
        print(json.dumps({"metric": nm, "host_us": round(host, 1), "total_us": round(total, 1)}), flush=True)
    # compute() per member (cache cleared each call) and per collection
    for name, m in list(cls.items(keep_base=True)) + list(reg.items(keep_base=True)):
        def fcomp(m=m):
            m._computed = None
            m.compute()
        host, total = timed(fcomp, n=50)
        print(json.dumps({"compute": name, "host_us": round(host, 1), "total_us": round(total, 1)}), flush=True)
    for nm, coll in (("collection_cls", cls), ("collection_reg", reg)):
        def fcc(coll=coll):
            for m in coll.values(copy_state=False):
                m._computed = None
            coll.compute()
        host, total = timed(fcc, n=50)
        print(json.dumps({"compute": nm, "host_us": round(host, 1), "total_us": round(total, 1)}), flush=True)
    print(json.dumps({"groups_cls": [list(v) for v in cls.compute_groups.values()],
                      "groups_reg": [list(v) for v in reg.compute_groups.values()]}))


if __name__ == "__main__":
    main()
