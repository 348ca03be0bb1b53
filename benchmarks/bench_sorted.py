"""Sort / scan kernel family vs the reference's formulations, on the same device.

Cases (one JSON line each; ``ours_ms`` = our public functional / metric compute, ``ref_ms`` = the reference's op
sequence re-expressed with plain torch ops in this process, since the reference itself is not importable here):

* binary AUROC / AP, 10^7 samples (reference: ``_binary_clf_curve`` argsort + distinct-value scan + cumsum, ROC /
  PR arrays, trapezoid -- ``F/classification/precision_recall_curve.py:28-80``, ``auroc.py:45-106``);
* multiclass AUROC, 10^6 x 100 classes (reference: Python loop over classes of the above);
* retrieval MAP, 10^6 documents / 10^4 queries (reference: sort by query, ``split`` sizes to host, Python loop over
  queries -- ``S/retrieval/base.py:147-190``; emulated on 1/10 of the queries and scaled);
* Spearman 10^7 (reference ``_rank_data``: ``torch.unique(return_inverse, return_counts)`` + cumsum);
* Kendall tau-b 10^6 (reference: all-pairs O(n^2) -- infeasible at 10^6; compared against our own host-side
  O(n log^2 n) torch formulation instead, reported as ``torch_knight_ms``).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402
from torchmetrics_amd import functional as F  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def ref_clf_curve(preds, target):
    desc = torch.argsort(preds, descending=True)
    preds, target = preds[desc], target[desc]
    distinct = torch.where(preds[1:] - preds[:-1])[0]
    idx = torch.nn.functional.pad(distinct, [0, 1], value=target.size(0) - 1)
    target = (target == 1).to(torch.long)
    tps = torch.cumsum(target * 1.0, dim=0)[idx]
    fps = 1 + idx - tps
    return fps, tps, preds[idx]


def ref_binary_auroc(preds, target):
    fps, tps, _ = ref_clf_curve(preds, target)
    tps = torch.cat([torch.zeros(1, device=tps.device), tps])
    fps = torch.cat([torch.zeros(1, device=fps.device), fps])
    if fps[-1] <= 0 or tps[-1] <= 0:  # reference warning checks (host reads)
        pass
    fpr, tpr = fps / fps[-1], tps / tps[-1]
    dx = fpr[1:] - fpr[:-1]
    direction = -1.0 if bool((dx < 0).any()) else 1.0  # reference _auc_compute direction check (host read)
    return torch.trapz(tpr, fpr) * direction


def ref_binary_ap(preds, target):
    fps, tps, _ = ref_clf_curve(preds, target)
    precision = tps / (tps + fps)
    recall = tps / tps[-1]
    precision = torch.cat([precision.flip(0), torch.ones(1, device=preds.device)])
    recall = torch.cat([recall.flip(0), torch.zeros(1, device=preds.device)])
    return -torch.sum((recall[1:] - recall[:-1]) * precision[:-1])


def ref_multiclass_auroc(preds, target, c):
    return torch.stack([ref_binary_auroc(preds[:, i], (target == i).long()) for i in range(c)]).mean()


def ref_retrieval_map(preds, target, indexes, max_queries=None):
    indexes, order = torch.sort(indexes)
    preds, target = preds[order], target[order]
    sizes = torch.bincount(indexes).cpu().tolist()
    sizes = [s for s in sizes if s]
    res = []
    for i, (p, t) in enumerate(zip(torch.split(preds, sizes), torch.split(target, sizes))):
        if max_queries is not None and i >= max_queries:
            break
        if not t.sum():
            res.append(torch.tensor(0.0, device=preds.device))
            continue
        t = t[torch.argsort(p, dim=-1, descending=True)]
        pos = torch.arange(1, len(t) + 1, device=t.device, dtype=torch.float32)[t > 0]
        res.append(torch.div(torch.arange(len(pos), device=pos.device, dtype=torch.float32) + 1, pos).mean())
    return torch.stack(res).mean()


def ref_rank(x):
    _, inverse, counts = torch.unique(x, sorted=True, return_inverse=True, return_counts=True)
    ranks = torch.cumsum(counts, dim=0)
    return ranks[inverse]


def ref_spearman(x, y):
    x, y = ref_rank(x).double(), ref_rank(y).double()
    xd, yd = x - x.mean(), y - y.mean()
    return (xd * yd).mean() / (xd.pow(2).mean().sqrt() * yd.pow(2).mean().sqrt())


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="run only the cases whose name contains this string")
    only = ap.parse_args().only
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []

    def want(name):
        return only in name

    n = 10**7
    p = torch.rand(n, device=dev, generator=g)
    t = (torch.rand(n, device=dev, generator=g) < p).long()
    from torchmetrics_amd import ops
    from torchmetrics_amd.functional.classification import _sorted

    if want("binary_auroc"):
      a, b = F.binary_auroc(p, t), ref_binary_auroc(p, t)
      out.append({"case": "binary_auroc n=1e7", "ours_ms": timeit(lambda: F.binary_auroc(p, t, validate_args=False)),
                "ref_ms": timeit(lambda: ref_binary_auroc(p, t)), "abs_diff": abs(float(a) - float(b)),
                "ours_validated_ms": timeit(lambda: F.binary_auroc(p, t)),
                "kernel_only_ms": timeit(lambda: _sorted.column_stats(p, t, ops.CLF_T_BINARY))})
    if want("binary_average_precision"):
      a, b = F.binary_average_precision(p, t), ref_binary_ap(p, t)
      out.append({"case": "binary_average_precision n=1e7", "ours_ms": timeit(lambda: F.binary_average_precision(p, t, validate_args=False)),
                "ref_ms": timeit(lambda: ref_binary_ap(p, t)), "abs_diff": abs(float(a) - float(b))})

    m, c = 10**6, 100
    pm = torch.randn(m, c, device=dev, generator=g).softmax(-1)
    tm_ = torch.randint(0, c, (m,), device=dev, generator=g)
    if want("multiclass_auroc"):
      a, b = F.multiclass_auroc(pm, tm_, c), ref_multiclass_auroc(pm, tm_, c)
      out.append({"case": "multiclass_auroc m=1e6 C=100", "ours_ms": timeit(lambda: F.multiclass_auroc(pm, tm_, c, validate_args=False), 3),
                "ref_ms": timeit(lambda: ref_multiclass_auroc(pm, tm_, c), 2), "abs_diff": abs(float(a) - float(b)),
                "kernel_only_ms": timeit(lambda: _sorted.column_stats(pm, tm_, ops.CLF_T_OVR), 3)})

    nd, nq = 10**6, 10**4
    pr = torch.rand(nd, device=dev, generator=g)
    tr = torch.randint(0, 2, (nd,), device=dev, generator=g)
    ir = torch.randint(0, nq, (nd,), device=dev, generator=g)
    metric = tm.retrieval.RetrievalMAP().to(dev)
    metric.update(pr, tr, ir)

    def ours_map():
        metric._computed = None
        return metric.compute()

    frac = 10
    if want("retrieval_map"):
      ref_ms = timeit(lambda: ref_retrieval_map(pr, tr, ir, nq // frac), 1) * frac
      out.append({"case": "retrieval_map n=1e6 queries=1e4", "ours_ms": timeit(ours_map, 5),
                "ref_ms": ref_ms, "ref_note": f"per-query loop timed on 1/{frac} of the queries, scaled",
                "abs_diff": abs(float(ours_map()) - float(ref_retrieval_map(pr, tr, ir)))})

    x = torch.randn(n, device=dev, generator=g)
    y = x + torch.randn(n, device=dev, generator=g)
    if want("spearman"):
      a, b = F.spearman_corrcoef(x, y), ref_spearman(x, y)
      out.append({"case": "spearman n=1e7", "ours_ms": timeit(lambda: F.spearman_corrcoef(x, y)),
                "ref_ms": timeit(lambda: ref_spearman(x, y)), "abs_diff": abs(float(a) - float(b))})

    nk = 10**6
    xk = torch.randn(nk, device=dev, generator=g, dtype=torch.float64)
    yk = (xk + torch.randn(nk, device=dev, generator=g, dtype=torch.float64)).round(decimals=1)
    from torchmetrics_amd.functional.regression import correlation as C

    def torch_knight():
        return C._pair_counts(xk.unsqueeze(1), yk.unsqueeze(1))

    if want("kendall"):
      out.append({"case": "kendall_tau_b n=1e6", "ours_ms": timeit(lambda: F.kendall_rank_corrcoef(xk, yk), 3),
                "torch_knight_ms": timeit(torch_knight, 1), "ref_ms": None,
                "ref_note": "reference is all-pairs O(n^2): 5e11 pairs, not run"})
    for o in out:
        if o.get("ref_ms"):
            o["speedup"] = round(o["ref_ms"] / o["ours_ms"], 2)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in o.items()}), flush=True)


if __name__ == "__main__":
    main()
