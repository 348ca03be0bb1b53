"""Score algebra on tp/fp/tn/fn shared by Accuracy / Precision / Recall / F-beta / Specificity / Hamming.

Parity with the reference ``_*_reduce`` functions (e.g. ``F/classification/accuracy.py:37-86``,
``precision_recall.py:37``, ``f_beta.py:37``, ``specificity.py:37``, ``hamming.py:37``): one table-driven
implementation instead of one function per metric.
"""
from typing import Callable, Dict, Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.compute import _adjust_weights_safe_divide, _safe_divide

_KIND_IDS = {"accuracy": 0, "hamming": 1, "precision": 2, "recall": 3, "specificity": 4, "fbeta": 5}
_AVG_IDS = {"micro": 0, "macro": 1, "weighted": 2, "none": 3}


def _sum_stats(x: Tensor, multidim_average: str) -> Tensor:
    return x.sum(dim=0 if multidim_average == "global" else 1)


def _score(kind: str, tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, multilabel: bool, beta: float) -> Tensor:
    if kind == "accuracy":
        return _safe_divide(tp + tn, tp + tn + fp + fn) if multilabel else _safe_divide(tp, tp + fn)
    if kind == "hamming":
        return 1 - (_safe_divide(tp + tn, tp + tn + fp + fn) if multilabel else _safe_divide(tp, tp + fn))
    if kind == "precision":
        return _safe_divide(tp, tp + fp)
    if kind == "recall":
        return _safe_divide(tp, tp + fn)
    if kind == "specificity":
        return _safe_divide(tn, tn + fp)
    if kind == "fbeta":
        b2 = beta**2
        return _safe_divide((1 + b2) * tp, (1 + b2) * tp + b2 * fn + fp)
    raise ValueError(kind)


def _binary_score(kind: str, tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor, beta: float) -> Tensor:
    if kind == "accuracy":
        return _safe_divide(tp + tn, tp + tn + fp + fn)
    if kind == "hamming":
        return 1 - _safe_divide(tp + tn, tp + fp + tn + fn)
    return _score(kind, tp, fp, tn, fn, False, beta)


def _stat_reduce(
    kind: str,
    tp: Tensor,
    fp: Tensor,
    tn: Tensor,
    fn: Tensor,
    average: Optional[str],
    multidim_average: str = "global",
    multilabel: bool = False,
    beta: float = 1.0,
) -> Tensor:
    """Reduce tp/fp/tn/fn to a score according to ``average`` (``binary``/``micro``/``macro``/``weighted``/``none``).

    ROCm int64 states take the single-launch fused reduction (``csrc/classification/stat_reduce.hip``)."""
    if tp.is_cuda and average != "binary" and tp.dtype == torch.int64:
        nd = tp.ndim
        shape = tp.shape
        if ((nd == 1 or (nd == 2 and multidim_average != "global")) and fp.shape == shape and tn.shape == shape
                and fn.shape == shape and fp.dtype == tn.dtype == fn.dtype == torch.int64):
            avg = _AVG_IDS[average if average is not None else "none"]
            if nd == 1:
                tp, fp, tn, fn = tp.reshape(1, -1), fp.reshape(1, -1), tn.reshape(1, -1), fn.reshape(1, -1)
            out = ops.stat_reduce(tp, fp, tn, fn, _KIND_IDS[kind], avg, multilabel, beta)
            if avg == 3:
                return out.view(shape)
            return out.view(()) if nd == 1 else out
    if average == "binary":
        return _binary_score(kind, tp, fp, tn, fn, beta)
    if average == "micro":
        tp, fp, tn, fn = (_sum_stats(x, multidim_average) for x in (tp, fp, tn, fn))
        if kind in ("accuracy", "hamming") and multilabel:
            return _binary_score(kind, tp, fp, tn, fn, beta)
        return _score(kind, tp, fp, tn, fn, False, beta)
    score = _score(kind, tp, fp, tn, fn, multilabel, beta)
    return _adjust_weights_safe_divide(score, average, multilabel, tp, fp, fn)


def _accuracy_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False):  # noqa: ANN001,ANN201
    return _stat_reduce("accuracy", tp, fp, tn, fn, average, multidim_average, multilabel)


def _precision_recall_reduce(stat, tp, fp, tn, fn, average, multidim_average="global", multilabel=False):  # noqa
    return _stat_reduce(stat, tp, fp, tn, fn, average, multidim_average, multilabel)


def _fbeta_reduce(tp, fp, tn, fn, beta, average, multidim_average="global", multilabel=False):  # noqa
    return _stat_reduce("fbeta", tp, fp, tn, fn, average, multidim_average, multilabel, beta)


def _specificity_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False):  # noqa
    return _stat_reduce("specificity", tp, fp, tn, fn, average, multidim_average, multilabel)


def _hamming_distance_reduce(tp, fp, tn, fn, average, multidim_average="global", multilabel=False):  # noqa
    return _stat_reduce("hamming", tp, fp, tn, fn, average, multidim_average, multilabel)
