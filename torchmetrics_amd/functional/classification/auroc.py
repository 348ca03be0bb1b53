"""Area under the ROC curve (reference ``F/classification/auroc.py:45-470``).

Unbinned multiclass / multilabel AUROC is computed for *all* columns at once from one segmented sort
(:func:`_batched_sorted_stats`): with scores sorted descending per column, every negative sample contributes the mean
of the true-positive counts just before and just after its tie group, which is exactly the trapezoid under the
tie-collapsed ROC curve.  The reference loops over classes, sorting and building each curve separately.
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.precision_recall_curve import (
    Thresholds,
    _binary_curve_state,
    _multiclass_curve_state,
    _multiclass_precision_recall_curve_arg_validation,
    _multilabel_curve_state,
    _multilabel_precision_recall_curve_arg_validation,
    _binary_precision_recall_curve_arg_validation,
    _task_dispatch,
)
from torchmetrics_amd.functional.classification.roc import (
    _binary_roc_compute,
    _multiclass_roc_compute,
    _multilabel_roc_compute,
)
from torchmetrics_amd.utilities.compute import _auc_compute_without_check, _safe_divide
from torchmetrics_amd.utilities.data import _bincount
from torchmetrics_amd.utilities.prints import rank_zero_warn


# ------------------------------------------------------------------------------------------- batched (unbinned)
def _batched_sorted_stats(scores: Tensor, pos: Tensor, valid: Optional[Tensor] = None):
    """Sort ``[M, K]`` scores per column (descending) and return tie-group statistics (fp64).

    Returns ``(pos_w, neg_w, tp_before, tp_after, fp_after, P, F)``: per sorted element its positive / negative weight,
    the cumulative TP count before its tie group and at its end, the cumulative FP count at its end, and the column
    totals.
    """
    if valid is not None:
        scores = torch.where(valid, scores, torch.full_like(scores, float("-inf")))
    s, order = torch.sort(scores, dim=0, descending=True)
    pos_w = torch.gather(pos.to(torch.float64), 0, order)
    neg_w = 1.0 - pos_w
    if valid is not None:
        v = torch.gather(valid.to(torch.float64), 0, order)
        pos_w, neg_w = pos_w * v, neg_w * v
    m = s.shape[0]
    tps, fps = pos_w.cumsum(0), neg_w.cumsum(0)
    idx = torch.arange(m, device=s.device).unsqueeze(1).expand_as(s)
    is_end = torch.ones_like(s, dtype=torch.bool)
    is_end[:-1] = s[1:] != s[:-1]
    is_start = torch.ones_like(s, dtype=torch.bool)
    is_start[1:] = is_end[:-1]
    # index of the group end at or after i: reverse running minimum over end positions
    end_idx = torch.where(is_end, idx, torch.full_like(idx, m)).flip(0).cummin(0).values.flip(0)
    start_idx = torch.where(is_start, idx, torch.full_like(idx, -1)).cummax(0).values
    tp_after = torch.gather(tps, 0, end_idx)
    fp_after = torch.gather(fps, 0, end_idx)
    before = (start_idx - 1).clamp(min=0)
    tp_before = torch.where(start_idx > 0, torch.gather(tps, 0, before), torch.zeros_like(tps))
    return pos_w, neg_w, tp_before, tp_after, fp_after, tps[-1], fps[-1]


def _batched_auroc(scores: Tensor, pos: Tensor, valid: Optional[Tensor] = None) -> Tensor:
    """Per-column ROC AUC of ``[M, K]`` scores; 0 for columns without positives or negatives (reference behaviour)."""
    if scores.shape[0] == 0:
        return torch.zeros(scores.shape[1], dtype=torch.float32, device=scores.device)
    pos_w, neg_w, tp_b, tp_a, _, p, f = _batched_sorted_stats(scores, pos, valid)
    area = (neg_w * (tp_a + tp_b)).sum(0) * 0.5
    denom = p * f
    res = torch.where(denom > 0, area / denom.clamp(min=1), torch.zeros_like(area))
    return res.to(torch.float32)


def _batched_average_precision(scores: Tensor, pos: Tensor, valid: Optional[Tensor] = None) -> Tensor:
    """Per-column step-wise AP; NaN for columns without positives (reference behaviour)."""
    if scores.shape[0] == 0:
        return torch.full((scores.shape[1],), float("nan"), dtype=torch.float32, device=scores.device)
    pos_w, _, _, tp_a, fp_a, p, _ = _batched_sorted_stats(scores, pos, valid)
    prec = tp_a / (tp_a + fp_a).clamp(min=1)
    num = torch.where(pos_w > 0, pos_w * prec, torch.zeros_like(prec)).sum(0)
    return (num / p).to(torch.float32)  # p == 0 -> nan


def _reduce_scores(
    res: Tensor, average: Optional[str], weights: Optional[Tensor], name: str = "Average precision"
) -> Tensor:
    if average is None or average == "none":
        return res
    if torch.isnan(res).any():
        rank_zero_warn(
            f"{name} score for one or more classes was `nan`. Ignoring these classes in {average}-average",
            UserWarning,
        )
    idx = ~torch.isnan(res)
    if average == "macro":
        return res[idx].mean()
    if average == "weighted" and weights is not None:
        w = _safe_divide(weights[idx], weights[idx].sum())
        return (res[idx] * w).sum()
    raise ValueError("Received an incompatible combinations of inputs to make reduction.")


def _fused_curve_score(state: Tensor, kind: int, average: Optional[str], name: str) -> Tensor:
    """Binned AUROC / AP on ROCm: one fused launch (``ops.curve_score``) instead of ~20 ops and two host syncs; the
    reference's nan warning costs one 4-byte read."""
    per_class, reduced, nan_flag = ops.curve_score(state, kind, average)
    if average is None or average == "none":
        return per_class
    if average not in ("macro", "weighted"):
        raise ValueError("Received an incompatible combinations of inputs to make reduction.")
    if bool(nan_flag.item()):
        rank_zero_warn(
            f"{name} score for one or more classes was `nan`. Ignoring these classes in {average}-average",
            UserWarning,
        )
    return reduced


def _reduce_auroc(
    fpr: Union[Tensor, List[Tensor]],
    tpr: Union[Tensor, List[Tensor]],
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    weights: Optional[Tensor] = None,
) -> Tensor:
    if isinstance(fpr, Tensor) and isinstance(tpr, Tensor):
        res = _auc_compute_without_check(fpr, tpr, 1.0, axis=1)
    else:
        res = torch.stack([_auc_compute_without_check(x, y, 1.0) for x, y in zip(fpr, tpr)])
    return _reduce_scores(res, average, weights)


# ------------------------------------------------------------------------------------------------------- binary
def _binary_auroc_arg_validation(
    max_fpr: Optional[float] = None, thresholds: Thresholds = None, ignore_index: Optional[int] = None
) -> None:
    _binary_precision_recall_curve_arg_validation(thresholds, ignore_index)
    if max_fpr is not None and not (isinstance(max_fpr, float) and 0 < max_fpr <= 1):
        raise ValueError(f"Arguments `max_fpr` should be a float in range (0, 1], but got: {max_fpr}")


def _binary_auroc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    thresholds: Optional[Tensor],
    max_fpr: Optional[float] = None,
    pos_label: int = 1,
) -> Tensor:
    fpr, tpr, _ = _binary_roc_compute(state, thresholds, pos_label)
    if max_fpr is None or max_fpr == 1 or fpr.sum() == 0 or tpr.sum() == 0:
        return _auc_compute_without_check(fpr, tpr, 1.0)
    # McClish-standardised partial AUC up to max_fpr (reference F/classification/auroc.py:82-106)
    max_area = torch.tensor(max_fpr, device=fpr.device)
    stop = torch.bucketize(max_area, fpr, out_int32=True, right=True)
    weight = (max_area - fpr[stop - 1]) / (fpr[stop] - fpr[stop - 1])
    interp_tpr = torch.lerp(tpr[stop - 1], tpr[stop], weight)
    tpr = torch.cat([tpr[:stop], interp_tpr.view(1)])
    fpr = torch.cat([fpr[:stop], max_area.view(1)])
    partial_auc = _auc_compute_without_check(fpr, tpr, 1.0)
    min_area = 0.5 * max_area**2
    return 0.5 * (1 + (partial_auc - min_area) / (max_area - min_area))


def binary_auroc(
    preds: Tensor,
    target: Tensor,
    max_fpr: Optional[float] = None,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary ROC AUC, optionally the standardised partial AUC up to ``max_fpr``."""
    if validate_args:
        _binary_auroc_arg_validation(max_fpr, thresholds, ignore_index)
    state, thr = _binary_curve_state(preds, target, thresholds, ignore_index, validate_args)
    return _binary_auroc_compute(state, thr, max_fpr)


# --------------------------------------------------------------------------------------------------- multiclass
def _multiclass_auroc_arg_validation(
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
    allowed_average = ("macro", "weighted", "none", None)
    if average not in allowed_average:
        raise ValueError(f"Expected argument `average` to be one of {allowed_average} but got {average}")


def _multiclass_auroc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Optional[Tensor] = None,
) -> Tensor:
    if isinstance(state, Tensor) and thresholds is not None:
        if state.is_cuda:
            return _fused_curve_score(state, ops.SCORE_AUROC, average, "AUROC")
        fpr, tpr, _ = _multiclass_roc_compute(state, num_classes, thresholds)
        return _reduce_auroc(fpr, tpr, average, weights=state[0][:, 1, :].sum(-1))
    preds, target = state
    pos = target.unsqueeze(1) == torch.arange(num_classes, device=target.device)
    res = _batched_auroc(preds, pos)
    return _reduce_scores(res, average, _bincount(target, minlength=num_classes).float())


def multiclass_auroc(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """One-vs-rest ROC AUC for multiclass tasks."""
    state, thr = _multiclass_curve_state(
        preds, target, num_classes, thresholds, None, ignore_index, validate_args,
        arg_validation=lambda: _multiclass_auroc_arg_validation(num_classes, average, thresholds, ignore_index),
    )
    return _multiclass_auroc_compute(state, num_classes, average, thr)


# --------------------------------------------------------------------------------------------------- multilabel
def _multilabel_auroc_arg_validation(
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]],
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
    allowed_average = ("micro", "macro", "weighted", "none", None)
    if average not in allowed_average:
        raise ValueError(f"Expected argument `average` to be one of {allowed_average} but got {average}")


def _multilabel_valid(target: Tensor, ignore_index: Optional[int]) -> Optional[Tensor]:
    return None if ignore_index is None else target != ignore_index


def _multilabel_auroc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]],
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
) -> Tensor:
    if isinstance(state, Tensor) and thresholds is not None:
        if average == "micro":
            return _binary_auroc_compute(state.sum(1), thresholds, max_fpr=None)
        if state.is_cuda:
            return _fused_curve_score(state, ops.SCORE_AUROC, average, "AUROC")
        fpr, tpr, _ = _multilabel_roc_compute(state, num_labels, thresholds, ignore_index)
        return _reduce_auroc(fpr, tpr, average, weights=state[0][:, 1, :].sum(-1))
    preds, target = state
    valid = _multilabel_valid(target, ignore_index)
    if average == "micro":
        res = _batched_auroc(preds.reshape(-1, 1), (target == 1).reshape(-1, 1),
                             None if valid is None else valid.reshape(-1, 1))
        return res[0]
    res = _batched_auroc(preds, target == 1, valid)
    return _reduce_scores(res, average, (target == 1).sum(dim=0).float())


def multilabel_auroc(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Per-label ROC AUC for multilabel tasks, reduced by ``average``."""
    state, thr = _multilabel_curve_state(
        preds, target, num_labels, thresholds, ignore_index, validate_args,
        arg_validation=lambda: _multilabel_auroc_arg_validation(num_labels, average, thresholds, ignore_index),
    )
    return _multilabel_auroc_compute(state, num_labels, average, thr, ignore_index)


def auroc(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Thresholds = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    max_fpr: Optional[float] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Optional[Tensor]:
    """Task wrapper over the binary / multiclass / multilabel AUROC."""
    return _task_dispatch(
        task,
        lambda: binary_auroc(preds, target, max_fpr, thresholds, ignore_index, validate_args),
        lambda: multiclass_auroc(preds, target, num_classes, average, thresholds, ignore_index, validate_args),
        lambda: multilabel_auroc(preds, target, num_labels, average, thresholds, ignore_index, validate_args),
        num_classes,
        num_labels,
    )
