"""Cohen's kappa (functional). Parity: reference ``F/classification/cohen_kappa.py:33-250``."""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.confusion_matrix import (
    _binary_confusion_matrix_arg_validation,
    _multiclass_confusion_matrix_arg_validation,
    binary_confusion_matrix,
    multiclass_confusion_matrix,
)
from torchmetrics_amd.utilities.enums import ClassificationTaskNoMultilabel

_ALLOWED_WEIGHTS = ("linear", "quadratic", "none", None)


def _cohen_kappa_reduce(confmat: Tensor, weights: Optional[str] = None) -> Tensor:
    """``1 - sum(W * O) / sum(W * E)`` with ``E`` the outer product of the marginals."""
    if ops.confmat_reducible(confmat) and weights in (None, "none", "linear", "quadratic"):
        return ops.confmat_reduce(confmat, ops.CM_KAPPA, weights=weights)  # one launch on ROCm
    cm = confmat if confmat.is_floating_point() else confmat.float()
    c = cm.shape[0]
    rows = cm.sum(dim=1, keepdim=True)
    cols = cm.sum(dim=0, keepdim=True)
    expected = rows @ cols / cols.sum()
    idx = torch.arange(c, dtype=cm.dtype, device=cm.device)
    diff = idx.unsqueeze(0) - idx.unsqueeze(1)
    if weights is None or weights == "none":
        w = 1.0 - torch.eye(c, dtype=cm.dtype, device=cm.device)
    elif weights == "linear":
        w = diff.abs()
    elif weights == "quadratic":
        w = diff.pow(2.0)
    else:
        raise ValueError(
            f"Received {weights} for argument ``weights`` but should be either None, 'linear' or 'quadratic'"
        )
    return 1 - (w * cm).sum() / (w * expected).sum()


def _check_weights(weights: Optional[str]) -> None:
    if weights not in _ALLOWED_WEIGHTS:
        raise ValueError(f"Expected argument `weight` to be one of {_ALLOWED_WEIGHTS}, but got {weights}.")


def _binary_cohen_kappa_arg_validation(threshold: float = 0.5, ignore_index: Optional[int] = None,
                                       weights: Optional[str] = None) -> None:
    _binary_confusion_matrix_arg_validation(threshold, ignore_index, normalize=None)
    _check_weights(weights)


def _multiclass_cohen_kappa_arg_validation(num_classes: int, ignore_index: Optional[int] = None,
                                           weights: Optional[str] = None) -> None:
    _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index, normalize=None)
    _check_weights(weights)


def binary_cohen_kappa(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    weights: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Cohen's kappa for binary tasks."""
    if validate_args:
        _binary_cohen_kappa_arg_validation(threshold, ignore_index, weights)
    cm = binary_confusion_matrix(preds, target, threshold, None, ignore_index, validate_args)
    return _cohen_kappa_reduce(cm, weights)


def multiclass_cohen_kappa(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    weights: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Cohen's kappa for multiclass tasks."""
    if validate_args:
        _multiclass_cohen_kappa_arg_validation(num_classes, ignore_index, weights)
    cm = multiclass_confusion_matrix(preds, target, num_classes, None, ignore_index, validate_args)
    return _cohen_kappa_reduce(cm, weights)


def cohen_kappa(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    weights: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching Cohen's kappa (binary / multiclass)."""
    task = ClassificationTaskNoMultilabel.from_str(task)
    if task == ClassificationTaskNoMultilabel.BINARY:
        return binary_cohen_kappa(preds, target, threshold, weights, ignore_index, validate_args)
    if task == ClassificationTaskNoMultilabel.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_cohen_kappa(preds, target, num_classes, weights, ignore_index, validate_args)
    raise ValueError(f"Not handled value: {task}")
