"""Matthews correlation coefficient (functional). Parity: reference ``F/classification/matthews_corrcoef.py:37-260``."""
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
from torchmetrics_amd.utilities.enums import ClassificationTask


def _matthews_corrcoef_reduce(confmat: Tensor) -> Tensor:
    """Multiclass MCC (Gorodkin's R_K) from a confusion matrix; multilabel matrices are summed to one 2x2 first."""
    cm = confmat.sum(0) if confmat.ndim == 3 else confmat
    if ops.confmat_reducible(cm):
        return ops.confmat_reduce(cm, ops.CM_MCC)  # one launch on ROCm, degenerate cases decided on the device
    binary = cm.numel() == 4
    if binary:
        tn, fp, fn, tp = (v for v in cm.reshape(-1))
        if tp + tn != 0 and fp + fn == 0:
            return torch.tensor(1.0, dtype=cm.dtype, device=cm.device)
        if tp + tn == 0 and fp + fn != 0:
            return torch.tensor(-1.0, dtype=cm.dtype, device=cm.device)
    t_k = cm.sum(dim=-1).float()
    p_k = cm.sum(dim=-2).float()
    correct = torch.trace(cm).float()
    total = cm.sum().float()
    numer = correct * total - (t_k * p_k).sum()
    denom = (total**2 - (p_k * p_k).sum()) * (total**2 - (t_k * t_k).sum())
    if denom == 0 and binary:
        # limit of MCC for degenerate 2x2 matrices (Chicco et al.), as in the reference
        a = tp + tn if (tp == 0 or tn == 0) else 0
        b = fp + fn if (fp == 0 or fn == 0) else 0
        eps = torch.tensor(torch.finfo(torch.float32).eps, dtype=torch.float32, device=cm.device)
        numer = torch.sqrt(eps) * (a - b)
        denom = (tp + fp + eps) * (tp + fn + eps) * (tn + fp + eps) * (tn + fn + eps)
    elif denom == 0:
        return torch.tensor(0, dtype=cm.dtype, device=cm.device)
    return numer / torch.sqrt(denom)


def binary_matthews_corrcoef(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _binary_confusion_matrix_arg_validation(threshold, ignore_index)
    return _matthews_corrcoef_reduce(binary_confusion_matrix(preds, target, threshold, None, ignore_index, validate_args))


def multiclass_matthews_corrcoef(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index)
    return _matthews_corrcoef_reduce(
        multiclass_confusion_matrix(preds, target, num_classes, None, ignore_index, validate_args)
    )


def multilabel_matthews_corrcoef(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    if validate_args:
        _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index)
    return _matthews_corrcoef_reduce(
        multilabel_confusion_matrix(preds, target, num_labels, threshold, None, ignore_index, validate_args)
    )


def matthews_corrcoef(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_matthews_corrcoef(preds, target, threshold, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_matthews_corrcoef(preds, target, num_classes, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_matthews_corrcoef(preds, target, num_labels, threshold, ignore_index, validate_args)
    raise ValueError(f"Not handled value: {task}")
