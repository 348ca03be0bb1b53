"""Precision and recall (functional). Parity: reference ``F/classification/precision_recall.py``."""
from typing import Optional

from torch import Tensor

from torchmetrics_amd.functional.classification._family import (
    _binary_family,
    _multiclass_family,
    _multilabel_family,
    _task_family,
)
from torchmetrics_amd.functional.classification._reductions import (  # noqa: F401
    _accuracy_reduce,
    _hamming_distance_reduce,
    _precision_recall_reduce,
    _specificity_reduce,
)


def binary_precision(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary precision (fused HIP stat-scores kernel on ROCm tensors)."""
    return _binary_family("precision", preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_precision(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
    top_k: int = 1,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass precision."""
    return _multiclass_family(
        "precision", preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_precision(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel precision."""
    return _multilabel_family(
        "precision", preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def precision(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[str] = "micro",
    multidim_average: str = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """precision for ``task`` in binary / multiclass / multilabel."""
    return _task_family(
        "precision", preds, target, task, threshold, num_classes, num_labels, average, multidim_average, top_k,
        ignore_index, validate_args,
    )


def binary_recall(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Binary recall (fused HIP stat-scores kernel on ROCm tensors)."""
    return _binary_family("recall", preds, target, threshold, multidim_average, ignore_index, validate_args)


def multiclass_recall(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
    top_k: int = 1,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multiclass recall."""
    return _multiclass_family(
        "recall", preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args
    )


def multilabel_recall(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Multilabel recall."""
    return _multilabel_family(
        "recall", preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args
    )


def recall(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    average: Optional[str] = "micro",
    multidim_average: str = "global",
    top_k: Optional[int] = 1,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """recall for ``task`` in binary / multiclass / multilabel."""
    return _task_family(
        "recall", preds, target, task, threshold, num_classes, num_labels, average, multidim_average, top_k,
        ignore_index, validate_args,
    )
