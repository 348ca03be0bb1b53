"""Area under the ROC curve (reference ``F/classification/auroc.py:45-470``).

Unbinned AUROC is computed for *all* columns at once by the sorted-curve kernels (``csrc/sort/clf_curve.hip``,
:mod:`._sorted`): with scores sorted descending per column, every tie run contributes ``neg_run * (tp_before +
pos_run / 2)``, which is exactly the trapezoid under the tie-collapsed ROC curve, and no curve is materialised.  The
reference loops over classes, sorting and building each curve separately.
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification import _sorted
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
from torchmetrics_amd.utils.deferred import warn_if


# ------------------------------------------------------------------------------------------- batched (unbinned)
def _column_auroc(preds: Tensor, target: Tensor, tmode: int, pos_label: int = 1,
                  ignore_index: Optional[int] = None) -> Tuple[Tensor, Tensor]:
    """Per-column ROC AUC (0 for columns without positives or negatives, as the reference) and the per-column
    positive counts, from one sorted-curve launch for all columns."""
    if preds.shape[0] == 0:
        k = 1 if preds.ndim == 1 else preds.shape[1]
        z = torch.zeros(k, dtype=torch.float32, device=preds.device)
        return z, z.clone()
    st = _sorted.column_stats(preds, target, tmode, pos_label, ignore_index)[0]
    return _sorted.auroc_from_stats(st), st[:, _sorted.P].to(torch.float32)


def _column_average_precision(preds: Tensor, target: Tensor, tmode: int, pos_label: int = 1,
                              ignore_index: Optional[int] = None) -> Tuple[Tensor, Tensor]:
    """Per-column step-wise AP (NaN without positives, as the reference) and the per-column positive counts."""
    if preds.shape[0] == 0:
        k = 1 if preds.ndim == 1 else preds.shape[1]
        return (torch.full((k,), float("nan"), dtype=torch.float32, device=preds.device),
                torch.zeros(k, dtype=torch.float32, device=preds.device))
    st = _sorted.column_stats(preds, target, tmode, pos_label, ignore_index)[0]
    return _sorted.ap_from_stats(st), st[:, _sorted.P].to(torch.float32)


def _reduce_scores(
    res: Tensor, average: Optional[str], weights: Optional[Tensor], name: str = "Average precision",
    may_be_nan: bool = True,
) -> Tensor:
    """macro / weighted reduction ignoring NaN classes, on the device (masked sums instead of boolean indexing).

    The reference's nan warning costs one 1-byte read; ``may_be_nan=False`` (AUROC: never NaN) skips it.
    """
    if average is None or average == "none":
        return res
    if average not in ("macro", "weighted") or (average == "weighted" and weights is None):
        raise ValueError("Received an incompatible combinations of inputs to make reduction.")
    nan = torch.isnan(res)
    if may_be_nan:
        warn_if(nan, f"{name} score for one or more classes was `nan`. Ignoring these classes in {average}-average")
    vals = torch.where(nan, torch.zeros_like(res), res)
    keep = (~nan).to(res.dtype)
    if average == "macro":
        return vals.sum() / keep.sum()
    w = torch.where(nan, torch.zeros_like(res), weights.to(res.dtype))
    return (vals * _safe_divide(w, w.sum())).sum()


def _fused_curve_score(state: Tensor, kind: int, average: Optional[str], name: str) -> Tensor:
    """Binned AUROC / AP on ROCm: one fused launch (``ops.curve_score``) instead of ~20 ops and two host syncs; the
    reference's nan warning costs one 4-byte read."""
    per_class, reduced, nan_flag = ops.curve_score(state, kind, average)
    if average is None or average == "none":
        return per_class
    if average not in ("macro", "weighted"):
        raise ValueError("Received an incompatible combinations of inputs to make reduction.")
    warn_if(nan_flag, f"{name} score for one or more classes was `nan`. Ignoring these classes in {average}-average")
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
    if thresholds is None and (max_fpr is None or max_fpr == 1):
        # whole-curve AUC straight from the sorted-run stats: no curve materialisation; the reference's
        # degenerate-curve warnings need the two totals (one 16-byte read)
        preds, target = state
        if preds.ndim > target.ndim:
            preds = preds[:, 0]
        if preds.numel():
            st = _sorted.column_stats(preds.reshape(-1), target.reshape(-1), ops.CLF_T_BINARY, pos_label)[0]
            n_pos, n_neg = st[0, :2].tolist()
            if n_neg <= 0:
                rank_zero_warn("No negative samples in targets, false positive value should be meaningless."
                               " Returning zero tensor in false positive score", UserWarning)
            if n_pos <= 0:
                rank_zero_warn("No positive samples in targets, true positive value should be meaningless."
                               " Returning zero tensor in true positive score", UserWarning)
            return _sorted.auroc_from_stats(st)[0]
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
    res, n_pos = _column_auroc(preds, target, ops.CLF_T_OVR)
    return _reduce_scores(res, average, n_pos, "AUROC", may_be_nan=False)


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
    if average == "micro":
        return _column_auroc(preds.reshape(-1), target.reshape(-1), ops.CLF_T_ELEM, 1, ignore_index)[0][0]
    res, n_pos = _column_auroc(preds, target, ops.CLF_T_ELEM, 1, ignore_index)
    return _reduce_scores(res, average, n_pos, "AUROC", may_be_nan=False)


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
