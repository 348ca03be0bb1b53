"""Jaccard index / IoU (functional). Parity: reference ``F/classification/jaccard.py:38-340``."""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.confusion_matrix import (
    _binary_confusion_matrix_arg_validation,
    _multiclass_confusion_matrix_arg_validation,
    _multilabel_confusion_matrix_arg_validation,
    binary_confusion_matrix,
    multiclass_confusion_matrix,
    multilabel_confusion_matrix,
)
from torchmetrics_amd.utilities.compute import _safe_divide
from torchmetrics_amd.utilities.enums import ClassificationTask

_ALLOWED_AVG = ("binary", "micro", "macro", "weighted", "none", None)


def _jaccard_index_reduce(confmat: Tensor, average: Optional[str], ignore_index: Optional[int] = None) -> Tensor:
    """IoU = tp / (tp + fp + fn) from a binary ``[2,2]``, multiclass ``[C,C]`` or multilabel ``[L,2,2]`` matrix."""
    if average not in _ALLOWED_AVG:
        raise ValueError(f"The `average` has to be one of {list(_ALLOWED_AVG)}, got {average}.")
    if average != "binary" and ops.confmat_reducible(confmat):
        return ops.confmat_reduce(confmat, ops.CM_JACCARD, average, ignore_index)  # one launch on ROCm
    cm = confmat.float()
    if average == "binary":
        return cm[1, 1] / (cm[0, 1] + cm[1, 0] + cm[1, 1])
    drop_ignored = ignore_index is not None and 0 <= ignore_index < cm.shape[0]
    multilabel = cm.ndim == 3
    if multilabel:
        tp = cm[:, 1, 1]
        union = cm[:, 1, 1] + cm[:, 0, 1] + cm[:, 1, 0]
    else:
        tp = torch.diagonal(cm)
        union = cm.sum(0) + cm.sum(1) - tp
    if average == "micro":
        tp = tp.sum()
        union = union.sum() - (union[ignore_index] if drop_ignored else 0.0)
    iou = _safe_divide(tp, union)
    if average in (None, "none", "micro"):
        return iou
    if average == "weighted":
        w = cm[:, 1, 1] + cm[:, 1, 0] if multilabel else cm.sum(1)
    else:
        w = torch.ones_like(iou)
        if drop_ignored:
            w[ignore_index] = 0.0
        if not multilabel:
            w = torch.where(cm.sum(1) + cm.sum(0) == 0, torch.zeros_like(w), w)
    return ((w * iou) / w.sum()).sum()


def _check_avg(average: Optional[str]) -> None:
    allowed = ("micro", "macro", "weighted", "none", None)
    if average not in allowed:
        raise ValueError(f"Expected argument `average` to be one of {allowed}, but got {average}.")


def binary_jaccard_index(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _binary_confusion_matrix_arg_validation(threshold, ignore_index)
    cm = binary_confusion_matrix(preds, target, threshold, None, ignore_index, validate_args)
    return _jaccard_index_reduce(cm, average="binary")


def multiclass_jaccard_index(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index)
        _check_avg(average)
    cm = multiclass_confusion_matrix(preds, target, num_classes, None, ignore_index, validate_args)
    return _jaccard_index_reduce(cm, average=average, ignore_index=ignore_index)


def multilabel_jaccard_index(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index)
        _check_avg(average)
    cm = multilabel_confusion_matrix(preds, target, num_labels, threshold, None, ignore_index, validate_args)
    return _jaccard_index_reduce(cm, average=average, ignore_index=ignore_index)


def jaccard_index(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[str] = "macro",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_jaccard_index(preds, target, threshold, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_jaccard_index(preds, target, num_classes, average, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_jaccard_index(preds, target, num_labels, threshold, average, ignore_index, validate_args)
    raise ValueError(f"Not handled value: {task}")
