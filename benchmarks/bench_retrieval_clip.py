"""Retrieval PR curve (``RetrievalPrecisionRecallCurve.compute``) and the CLIP metric math: ours vs an op-for-op
emulation of the reference paths.  One JSON line per case.

* PR curve: 200k documents in 2000 queries of 100; ours = one (query, score) sort + one wave-per-query curve kernel
  (``csrc/sort/retrieval.hip``); reference = ``S/retrieval/precision_recall_curve.py:190-236`` (sort by query, group
  sizes to the host, per-query ``F/retrieval/precision_recall_curve.py:87-99``: topk, pad, cumsum, two divides).
* CLIPScore math: ``100 * cos`` of 4096 (image, caption) embedding pairs, D = 768 (``F/multimodal/clip_score.py``:
  two normalisations + product + sum) vs ``paired_cosine``.
* CLIP-IQA: 4096 images x 16 prompt pairs (``F/multimodal/clip_iqa.py:171-178``: GEMM + softmax) vs
  ``prompt_pair_prob``.
"""
import argparse
import json
import os
import sys
import time

import torch
from torch.nn.functional import pad

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchmetrics_amd as tm  # noqa: E402
from torchmetrics_amd import ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out


def ref_pr_curve(preds, target, indexes, max_k=None):
    indexes, order = torch.sort(indexes)
    preds, target = preds[order], target[order]
    sizes = torch.bincount(indexes).cpu().tolist()
    sizes = [s for s in sizes if s]
    max_k = max(sizes) if max_k is None else max_k
    ps, rs = [], []
    for p, t in zip(torch.split(preds, sizes), torch.split(target, sizes)):
        if not t.sum():
            ps.append(torch.zeros(max_k, device=p.device))
            rs.append(torch.zeros(max_k, device=p.device))
            continue
        topk = torch.arange(1, max_k + 1, device=p.device)
        rel = t[p.topk(min(max_k, p.shape[-1]), dim=-1)[1]].float()
        rel = torch.cumsum(pad(rel, (0, max(0, max_k - len(rel))), "constant", 0.0), dim=0)
        rs.append(rel / t.sum())
        ps.append(rel / topk)
    return torch.stack(ps).mean(0), torch.stack(rs).mean(0)


def ref_clip(img, txt):
    img = img / img.norm(p=2, dim=-1, keepdim=True)
    txt = txt / txt.norm(p=2, dim=-1, keepdim=True)
    return 100 * (img * txt).sum(dim=-1)


def ref_iqa(img, anchors):
    logits = 100 * img @ anchors.t()
    return logits.reshape(logits.shape[0], -1, 2).softmax(-1)[:, :, 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ours-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    n_q, per = 2000, 100
    idx = torch.arange(n_q, device=dev).repeat_interleave(per)
    idx = idx[torch.randperm(idx.numel(), device=dev, generator=g)]
    preds = torch.rand(idx.numel(), device=dev, generator=g)
    target = torch.rand(idx.numel(), device=dev, generator=g) > 0.8
    m = tm.retrieval.RetrievalPrecisionRecallCurve().to(dev)
    m.update(preds, target, idx)

    def ours_pr():
        m._computed = None
        return m.compute()

    t_ours, (p1, r1, _) = timed(ours_pr)
    row = {"case": "retrieval_pr_curve", "docs": idx.numel(), "queries": n_q, "ours_ms": round(t_ours, 3)}
    if not args.ours_only:
        t_ref, (p2, r2) = timed(lambda: ref_pr_curve(preds, target, idx), reps=2)
        row.update(ref_ms=round(t_ref, 2), speedup=round(t_ref / t_ours, 1),
                   max_abs_diff=float(torch.maximum((p1 - p2).abs().max(), (r1 - r2).abs().max())))
    print(json.dumps(row), flush=True)

    n, d = 4096, 768
    img = torch.randn(n, d, device=dev, generator=g)
    txt = torch.randn(n, d, device=dev, generator=g)
    t_ours, s1 = timed(lambda: ops.paired_cosine(img, txt, 100.0), reps=50)
    row = {"case": "clip_score_math", "pairs": n, "dim": d, "ours_us": round(t_ours * 1e3, 1)}
    if not args.ours_only:
        t_ref, s2 = timed(lambda: ref_clip(img, txt), reps=50)
        row.update(ref_us=round(t_ref * 1e3, 1), speedup=round(t_ref / t_ours, 2),
                   max_abs_diff=float((s1 - s2).abs().max()))
    print(json.dumps(row), flush=True)

    imgn = img / img.norm(dim=-1, keepdim=True)
    anchors = torch.randn(32, d, device=dev, generator=g)
    anchors = anchors / anchors.norm(dim=-1, keepdim=True)
    t_ours, q1 = timed(lambda: ops.prompt_pair_prob(imgn, anchors, 100.0), reps=50)
    row = {"case": "clip_iqa_math", "images": n, "prompt_pairs": 16, "ours_us": round(t_ours * 1e3, 1)}
    if not args.ours_only:
        t_ref, q2 = timed(lambda: ref_iqa(imgn, anchors), reps=50)
        row.update(ref_us=round(t_ref * 1e3, 1), speedup=round(t_ref / t_ours, 2),
                   max_abs_diff=float((q1 - q2).abs().max()))
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
