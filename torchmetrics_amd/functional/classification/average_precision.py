"""Average precision (reference ``F/classification/average_precision.py:43-420``).

Binned: from the HIP multi-threshold confusion matrices.  Unbinned multiclass / multilabel: all columns in one
sorted-curve launch (``csrc/sort/clf_curve.hip`` via
:func:`~torchmetrics_amd.functional.classification.auroc._column_average_precision`).
"""
from typing import List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.auroc import (
    _column_average_precision,
    _fused_curve_score,
    _multilabel_valid,
    _reduce_scores,
)
from torchmetrics_amd.functional.classification.precision_recall_curve import (
    Thresholds,
    _binary_curve_state,
    _binary_precision_recall_curve_compute,
    _multiclass_curve_state,
    _multiclass_precision_recall_curve_arg_validation,
    _multiclass_precision_recall_curve_compute,
    _multilabel_curve_state,
    _multilabel_precision_recall_curve_arg_validation,
    _multilabel_precision_recall_curve_compute,
    _task_dispatch,
)
from torchmetrics_amd.utilities.data import _bincount


def _reduce_average_precision(
    precision: Union[Tensor, List[Tensor]],
    recall: Union[Tensor, List[Tensor]],
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    weights: Optional[Tensor] = None,
) -> Tensor:
    if isinstance(precision, Tensor) and isinstance(recall, Tensor):
        res = -torch.sum((recall[:, 1:] - recall[:, :-1]) * precision[:, :-1], 1)
    else:
        res = torch.stack([-torch.sum((r[1:] - r[:-1]) * p[:-1]) for p, r in zip(precision, recall)])
    return _reduce_scores(res, average, weights)


def _binary_average_precision_compute(state: Union[Tensor, Tuple[Tensor, Tensor]], thresholds: Optional[Tensor]) -> Tensor:
    if not isinstance(state, Tensor) or thresholds is None:
        preds, target = state
        if preds.ndim > target.ndim:
            preds = preds[:, 0]
        return _column_average_precision(preds.reshape(-1), target.reshape(-1), ops.CLF_T_BINARY)[0][0]
    precision, recall, _ = _binary_precision_recall_curve_compute(state, thresholds)
    return -torch.sum((recall[1:] - recall[:-1]) * precision[:-1])


def binary_average_precision(
    preds: Tensor,
    target: Tensor,
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary average precision (step-wise area under the PR curve)."""
    state, thr = _binary_curve_state(preds, target, thresholds, ignore_index, validate_args)
    return _binary_average_precision_compute(state, thr)


def _multiclass_average_precision_arg_validation(
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multiclass_precision_recall_curve_arg_validation(num_classes, thresholds, ignore_index)
    allowed_average = ("macro", "weighted", "none", None)
    if average not in allowed_average:
        raise ValueError(f"Expected argument `average` to be one of {allowed_average} but got {average}")


def _multiclass_average_precision_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Optional[Tensor] = None,
) -> Tensor:
    if isinstance(state, Tensor) and thresholds is not None:
        if state.is_cuda:
            return _fused_curve_score(state, ops.SCORE_AP, average, "Average precision")
        precision, recall, _ = _multiclass_precision_recall_curve_compute(state, num_classes, thresholds)
        return _reduce_average_precision(precision, recall, average, weights=state[0][:, 1, :].sum(-1))
    preds, target = state
    res, n_pos = _column_average_precision(preds, target, ops.CLF_T_OVR)
    return _reduce_scores(res, average, n_pos)


def multiclass_average_precision(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """One-vs-rest average precision for multiclass tasks."""
    state, thr = _multiclass_curve_state(
        preds, target, num_classes, thresholds, None, ignore_index, validate_args,
        arg_validation=lambda: _multiclass_average_precision_arg_validation(num_classes, average, thresholds,
                                                                            ignore_index),
    )
    return _multiclass_average_precision_compute(state, num_classes, average, thr)


def _multilabel_average_precision_arg_validation(
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]],
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
) -> None:
    _multilabel_precision_recall_curve_arg_validation(num_labels, thresholds, ignore_index)
    allowed_average = ("micro", "macro", "weighted", "none", None)
    if average not in allowed_average:
        raise ValueError(f"Expected argument `average` to be one of {allowed_average} but got {average}")


def _multilabel_average_precision_compute(
    state: Union[Tensor, Tuple[Tensor, Tensor]],
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]],
    thresholds: Optional[Tensor],
    ignore_index: Optional[int] = None,
) -> Tensor:
    if isinstance(state, Tensor) and thresholds is not None:
        if average == "micro":
            return _binary_average_precision_compute(state.sum(1), thresholds)
        if state.is_cuda:
            return _fused_curve_score(state, ops.SCORE_AP, average, "Average precision")
        precision, recall, _ = _multilabel_precision_recall_curve_compute(state, num_labels, thresholds, ignore_index)
        return _reduce_average_precision(precision, recall, average, weights=state[0][:, 1, :].sum(-1))
    preds, target = state
    if average == "micro":
        return _column_average_precision(preds.reshape(-1), target.reshape(-1), ops.CLF_T_ELEM, 1, ignore_index)[0][0]
    res, n_pos = _column_average_precision(preds, target, ops.CLF_T_ELEM, 1, ignore_index)
    return _reduce_scores(res, average, n_pos)


def multilabel_average_precision(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    average: Optional[Literal["micro", "macro", "weighted", "none"]] = "macro",
    thresholds: Thresholds = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Per-label average precision for multilabel tasks, reduced by ``average``."""
    state, thr = _multilabel_curve_state(
        preds, target, num_labels, thresholds, ignore_index, validate_args,
        arg_validation=lambda: _multilabel_average_precision_arg_validation(num_labels, average, thresholds,
                                                                            ignore_index),
    )
    return _multilabel_average_precision_compute(state, num_labels, average, thr, ignore_index)


def average_precision(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass", "multilabel"],
    thresholds: Thresholds = None,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[Literal["macro", "weighted", "none"]] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Optional[Tensor]:
    """Task wrapper over the binary / multiclass / multilabel average precision."""
    return _task_dispatch(
        task,
        lambda: binary_average_precision(preds, target, thresholds, ignore_index, validate_args),
        lambda: multiclass_average_precision(
            preds, target, num_classes, average, thresholds, ignore_index, validate_args
        ),
        lambda: multilabel_average_precision(preds, target, num_labels, average, thresholds, ignore_index,
                                             validate_args),
        num_classes,
        num_labels,
    )
