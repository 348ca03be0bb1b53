"""Sorted-curve statistics for every unbinned (``thresholds=None``) classification curve metric.

One call of :func:`torchmetrics_amd.ops.clf_curve` (``csrc/sort/clf_curve.hip`` on ROCm: packed-key radix sort +
tie-run scan, 5 launches whatever the number of classes) yields, per segment (class / label / sample row):
``P``, ``N`` (positive / negative weight), the trapezoid ROC area, the step-AP sum, the coverage rank and the number of
distinct thresholds, plus -- on request -- the compacted ``_binary_clf_curve`` of every segment.  The reference builds
these with a Python loop over classes, one ``argsort`` + ``cumsum`` + boolean indexing chain each
(``F/classification/precision_recall_curve.py:28-80``, ``auroc.py:45-106``, ``average_precision.py:43-80``).

Nothing here synchronises with the host except :func:`split_curves` / :func:`roc_curves` / :func:`pr_curves`, whose
variable-length outputs need the counts.  The last two build every segment's final curve in one ``[S, N + 1]``
epilogue (a handful of launches whatever ``S``) and hand out per-segment views of it; the reference runs its
``cat`` / divide / flip chain once per class (``F/classification/roc.py:107-112``,
``F/classification/precision_recall_curve.py:356-371``).
"""
import warnings
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops

P, N, AREA, AP, COV, NRUNS = 0, 1, 2, 3, 4, 6


def _seg_args(scores: Tensor) -> Tuple[int, int, int, int]:
    """``[M]`` -> one segment; ``[M, S]`` -> ``S`` column segments."""
    if scores.ndim == 1:
        return 1, scores.shape[0], 0, scores.stride(0)
    return scores.shape[1], scores.shape[0], scores.stride(1), scores.stride(0)


def column_stats(scores: Tensor, target: Tensor, tmode: int, pos_label: int = 1, ignore_index: Optional[int] = None,
                 emit: int = 0, weights: Optional[Tensor] = None) -> list:
    """Stats of the columns of ``scores`` ``[M, S]`` (or ``[M]``).

    ``tmode``: ``ops.CLF_T_BINARY`` (``target [M]`` vs ``pos_label``), ``ops.CLF_T_OVR`` (``target [M]`` class ids),
    ``ops.CLF_T_ELEM`` (``target`` shaped like ``scores``; must share its strides).
    """
    if not scores.is_contiguous():
        scores = scores.contiguous()
    if tmode == ops.CLF_T_ELEM:
        target = target.reshape(scores.shape).contiguous()
    else:
        target = target.contiguous()
    s, m, seg_stride, elem_stride = _seg_args(scores)
    return ops.clf_curve(scores, target, s, m, seg_stride, elem_stride, tmode, pos_label, ignore_index, weights, emit)


def row_stats(scores: Tensor, target: Tensor) -> Tensor:
    """Stats of the rows of ``scores`` ``[N, L]`` (label-ranking metrics): one segment per sample."""
    scores, target = scores.contiguous(), target.contiguous()
    n, l = scores.shape
    return ops.clf_curve(scores, target, n, l, l, 1, ops.CLF_T_ELEM)[0]


def auroc_from_stats(st: Tensor) -> Tensor:
    """Tie-aware trapezoid ROC AUC per segment; 0 when a segment lacks positives or negatives (reference)."""
    denom = st[:, P] * st[:, N]
    return torch.where(denom > 0, st[:, AREA] / torch.where(denom > 0, denom, torch.ones_like(denom)),
                       torch.zeros_like(denom)).to(torch.float32)


def ap_from_stats(st: Tensor) -> Tensor:
    """Step-wise average precision per segment; NaN without positives (reference)."""
    return (st[:, AP] / st[:, P]).to(torch.float32)


def split_curves(out: list, dtype: torch.dtype) -> Tuple[List[Tensor], List[Tensor], List[Tensor], List[List[float]]]:
    """Per-segment ``(fps, tps, thresholds)`` (descending thresholds), as ``_binary_clf_curve`` returns them, plus the
    host copy of the stats rows (``P``, ``N``, ...: callers decide the reference's degenerate-curve warnings from it).

    One host read: the ``[S, 8]`` stats (number of distinct thresholds of every segment).
    """
    st, fps, tps, thr = out[0], out[1], out[2], out[3]
    host = st.tolist()
    counts = [int(r[NRUNS]) for r in host]
    fps32, tps32, thr_c = fps.to(torch.float32), tps.to(torch.float32), thr.to(dtype)
    return ([fps32[i, :c] for i, c in enumerate(counts)], [tps32[i, :c] for i, c in enumerate(counts)],
            [thr_c[i, :c] for i, c in enumerate(counts)], host)


def _counts(st: Tensor) -> Tuple[List[List[float]], List[int], Tensor]:
    host = st.tolist()
    return host, [int(r[NRUNS]) for r in host], st[:, NRUNS].to(torch.long).unsqueeze(1)


def roc_curves(out: list, dtype: torch.dtype, warn=None) -> Tuple[List[Tensor], List[Tensor], List[Tensor]]:
    """Per-segment ``(fpr, tpr, thresholds)`` of ``_binary_roc_compute`` (a leading ``(0, 0, 1)`` point; a rate is
    zero, with the reference's warning, when its segment has no negatives / positives), as views of three
    ``[S, N + 1]`` buffers.  ``warn(message)`` defaults to :func:`warnings.warn`."""
    st, fps, tps, thr = out[0], out[1], out[2], out[3]
    host, counts, c = _counts(st)
    fps = torch.nn.functional.pad(fps.to(torch.float32), (1, 0))
    tps = torch.nn.functional.pad(tps.to(torch.float32), (1, 0))
    thr = torch.nn.functional.pad(thr.to(dtype), (1, 0), value=1.0)
    fden, tden = fps.gather(1, c), tps.gather(1, c)  # the last point: every negative / positive
    fpr = torch.where(fden > 0, fps / fden, torch.zeros((), dtype=fps.dtype, device=fps.device))
    tpr = torch.where(tden > 0, tps / tden, torch.zeros((), dtype=tps.dtype, device=tps.device))
    warn = warn or (lambda msg: warnings.warn(msg, UserWarning, stacklevel=3))
    for r in host:
        if r[N] <= 0:
            warn("No negative samples in targets, false positive value should be meaningless."
                 " Returning zero tensor in false positive score")
        if r[P] <= 0:
            warn("No positive samples in targets, true positive value should be meaningless."
                 " Returning zero tensor in true positive score")
    # a degenerate rate is `zeros_like(thresholds)` in the reference: the thresholds' dtype
    zero = torch.zeros_like(thr) if thr.dtype != torch.float32 else None
    fl = [fpr[i, : k + 1] if zero is None or r[N] > 0 else zero[i, : k + 1] for i, (k, r) in enumerate(zip(counts, host))]
    tl = [tpr[i, : k + 1] if zero is None or r[P] > 0 else zero[i, : k + 1] for i, (k, r) in enumerate(zip(counts, host))]
    return fl, tl, [thr[i, : k + 1] for i, k in enumerate(counts)]


def pr_curves(out: list, dtype: torch.dtype) -> Tuple[List[Tensor], List[Tensor], List[Tensor]]:
    """Per-segment ``(precision, recall, thresholds)`` of ``_binary_precision_recall_curve_compute`` (ascending
    thresholds, the ``(1, 0)`` end point appended), as views of three ``[S, N + 1]`` / ``[S, N]`` buffers: every row
    is reversed by one gather over its own length."""
    st, fps, tps, thr = out[0], out[1], out[2], out[3]
    _, counts, c = _counts(st)
    s, n = tps.shape
    dev = tps.device
    if n == 0:
        e = torch.zeros(s, 0, dtype=dtype, device=dev)
        one = torch.ones(s, 1, dtype=torch.float32, device=dev)
        return [one[i] for i in range(s)], [torch.zeros_like(one[i]) for i in range(s)], [e[i] for i in range(s)]
    j = torch.arange(n + 1, device=dev)
    idx = (c - 1 - j).clamp(min=0)
    tp, fp = tps.to(torch.float32), fps.to(torch.float32)
    tpf, fpf = tp.gather(1, idx), fp.gather(1, idx)
    end = j == c
    one = torch.ones((), dtype=torch.float32, device=dev)
    precision = torch.where(end, one, tpf / (tpf + fpf))
    recall = torch.where(end, torch.zeros_like(one), tpf / tp.gather(1, (c - 1).clamp(min=0)))
    thr_f = thr.to(dtype).gather(1, idx[:, :n])
    return ([precision[i, : k + 1] for i, k in enumerate(counts)],
            [recall[i, : k + 1] for i, k in enumerate(counts)], [thr_f[i, :k] for i, k in enumerate(counts)])
