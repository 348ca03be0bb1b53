"""Receiver operating characteristic curves (reference ``F/classification/roc.py:40-420``).

Binned states come from the HIP multi-threshold histogram (see ``precision_recall_curve``); unbinned curves from
one descending sort per column.
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.classification.precision_recall_curve import (
    _macro_average_curve,
    Thresholds,
    _binary_clf_curve,
    _clf_curves,
    _binary_curve_state,
    _multiclass_curve_state,
    _multilabel_curve_state,
    _multilabel_masked_column,
    _task_dispatch,
)
from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification import _sorted
from torchmetrics_amd.utilities.compute import _safe_divide
from torchmetrics_amd.utilities.prints import rank_zero_warn


def _rates_from_confmat(state: Tensor) -> Tuple[Tensor, Tensor]:
    tps, fps, fns, tns = state[..., 1, 1], state[..., 0, 1], state[..., 1, 0], state[..., 0, 0]
    return _safe_divide(fps, fps + tns), _safe_divide(tps, tps + fns)


def _clf_roc_curves(preds: Tensor, target: Tensor, tmode: int,
                    ignore_index: Optional[int] = None) -> Tuple[List[Tensor], List[Tensor], List[Tensor]]:
    """Every column's ROC curve from one sorted-curve launch and one ``[S, N + 1]`` epilogue; the per-class tensors
    are views of it (``_sorted.roc_curves``)."""
    out = _sorted.column_stats(preds, target, tmode, 1, ignore_index, ops.EMIT_CURVE)
    return _sorted.roc_curves(out, preds.dtype, warn=lambda msg: rank_zero_warn(msg, UserWarning))


def _binary_roc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    thresholds: Optional[Tensor],
    pos_label: int = 1,
) -> Tuple[Tensor, Tensor, Tensor]:
    if isinstance(state, Tensor) and thresholds is not None:
        fpr, tpr = _rates_from_confmat(state)
        return fpr.flip(0), tpr.flip(0), thresholds.flip(0)
    preds, target = state[0], state[1]
    if preds.ndim > target.ndim:
        preds = preds[:, 0]
    if preds.numel() == 0:
        fps, tps, thres = _binary_clf_curve(preds=preds, target=target, pos_label=pos_label)
        return _roc_from_clf(fps, tps, thres, 0.0, 0.0)
    fps, tps, thres, host = _clf_curves(preds.reshape(-1), target.reshape(-1), ops.CLF_T_BINARY, pos_label)
    return _roc_from_clf(fps[0], tps[0], thres[0], host[0][1], host[0][0])


def _roc_from_clf(fps: Tensor, tps: Tensor, thres: Tensor, n_neg: float, n_pos: float) -> Tuple[Tensor, Tensor, Tensor]:
    """ROC points from one ``_binary_clf_curve``; ``n_neg`` / ``n_pos`` are host totals (no device read here)."""
    tps = torch.cat([torch.zeros(1, dtype=tps.dtype, device=tps.device), tps])
    fps = torch.cat([torch.zeros(1, dtype=fps.dtype, device=fps.device), fps])
    thres = torch.cat([torch.ones(1, dtype=thres.dtype, device=thres.device), thres])
    if n_neg <= 0:
        rank_zero_warn(
            "No negative samples in targets, false positive value should be meaningless."
            " Returning zero tensor in false positive score",
            UserWarning,
        )
        fpr = torch.zeros_like(thres)
    else:
        fpr = fps / fps[-1]
    if n_pos <= 0:
        rank_zero_warn(
            "No positive samples in targets, true positive value should be meaningless."
            " Returning zero tensor in true positive score",
            UserWarning,
        )
        tpr = torch.zeros_like(thres)
    else:
        tpr = tps / tps[-1]
    return fpr, tpr, thres


def binary_roc(
    preds: Tensor,
    target: Tensor,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tuple[Tensor, Tensor, Tensor]:
    """``(fpr, tpr, thresholds)`` for binary tasks; thresholds descending."""
    state, thr = _binary_curve_state(preds, target, thresholds, ignore_index, validate_args)
    return _binary_roc_compute(state, thr)


def _multiclass_roc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_classes: int,
    thresholds: Optional[Tensor],
    average: Optional[Literal["micro", "macro"]] = None,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    if average == "micro":
        return _binary_roc_compute(state, thresholds, pos_label=1)
    if isinstance(state, Tensor) and thresholds is not None:
        fpr, tpr = _rates_from_confmat(state)
        fpr, tpr, thres = fpr.flip(0).T, tpr.flip(0).T, thresholds.flip(0)
        tensor_state = True
    else:
        fpr_list, tpr_list, thres_list = _clf_roc_curves(state[0], state[1], ops.CLF_T_OVR)
        tensor_state = False
    if average == "macro":
        if tensor_state:
            return _macro_average_curve(fpr, tpr, thres.repeat(num_classes), descending=True)
        return _macro_average_curve(fpr_list, tpr_list, torch.cat(thres_list), descending=True)
    if tensor_state:
        return fpr, tpr, thres
    return fpr_list, tpr_list, thres_list


def multiclass_roc(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    thresholds: Thresholds = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """One-vs-rest ROC curves for multiclass tasks."""
    state, thr = _multiclass_curve_state(preds, target, num_classes, thresholds, average, ignore_index, validate_args)
    return _multiclass_roc_compute(state, num_classes, thr, average)


def _multilabel_roc_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_labels: int,
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    if isinstance(state, Tensor) and thresholds is not None:
        fpr, tpr = _rates_from_confmat(state)
        return fpr.flip(0).T, tpr.flip(0).T, thresholds.flip(0)
    return _clf_roc_curves(state[0], state[1], ops.CLF_T_ELEM, ignore_index)


def multilabel_roc(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """Per-label ROC curves for multilabel tasks."""
    state, thr = _multilabel_curve_state(preds, target, num_labels, thresholds, ignore_index, validate_args)
    return _multilabel_roc_compute(state, num_labels, thr, ignore_index)


def roc(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Thresholds = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["micro", "macro"]] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Union[Tuple[Tensor, Tensor, Tensor], Tuple[List[Tensor], List[Tensor], List[Tensor]]]:
    """Task wrapper over the binary / multiclass / multilabel ROC."""
    return _task_dispatch(
        task,
        lambda: binary_roc(preds, target, thresholds, ignore_index, validate_args),
        lambda: multiclass_roc(preds, target, num_classes, thresholds, average, ignore_index, validate_args),
        lambda: multilabel_roc(preds, target, num_labels, thresholds, ignore_index, validate_args),
        num_classes,
        num_labels,
    )
