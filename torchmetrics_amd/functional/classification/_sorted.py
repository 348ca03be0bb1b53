"""Sorted-curve statistics for every unbinned (``thresholds=None``) classification curve metric.

One call of :func:`torchmetrics_amd.ops.clf_curve` (``csrc/sort/clf_curve.hip`` on ROCm: packed-key radix sort +
tie-run scan, 5 launches whatever the number of classes) yields, per segment (class / label / sample row):
``P``, ``N`` (positive / negative weight), the trapezoid ROC area, the step-AP sum, the coverage rank and the number of
distinct thresholds, plus -- on request -- the compacted ``_binary_clf_curve`` of every segment.  The reference builds
these with a Python loop over classes, one ``argsort`` + ``cumsum`` + boolean indexing chain each
(``F/classification/precision_recall_curve.py:28-80``, ``auroc.py:45-106``, ``average_precision.py:43-80``).

Nothing here synchronises with the host except :func:`split_curves`, whose variable-length outputs need the counts.
"""
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
