"""Shared driver for the functional stat-score family (one fused kernel + the score algebra of ``_reductions``)."""
from typing import Optional

from torch import Tensor

from torchmetrics_amd.functional.classification._reductions import _stat_reduce
from torchmetrics_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_tensor_validation,
    _binary_stat_scores_update,
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_tensor_validation,
    _multiclass_stat_scores_update,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_tensor_validation,
    _multilabel_stat_scores_update,
)
from torchmetrics_amd.utilities.enums import ClassificationTask


def _check_beta(beta: float) -> None:
    if not (isinstance(beta, float) and beta > 0):
        raise ValueError(f"Expected argument `beta` to be a float larger than 0, but got {beta}.")


def _binary_family(
    kind: str,
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
    beta: float = 1.0,
) -> Tensor:
    if validate_args:
        if kind == "fbeta":
            _check_beta(beta)
        _binary_stat_scores_arg_validation(threshold, multidim_average, ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, multidim_average, ignore_index)
    tp, fp, tn, fn = _binary_stat_scores_update(preds, target, threshold, multidim_average, ignore_index, validate_args)
    return _stat_reduce(kind, tp, fp, tn, fn, "binary", multidim_average, beta=beta)


def _multiclass_family(
    kind: str,
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    average: Optional[str] = "macro",
    top_k: int = 1,
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
    beta: float = 1.0,
) -> Tensor:
    if validate_args:
        if kind == "fbeta":
            _check_beta(beta)
        _multiclass_stat_scores_arg_validation(num_classes, top_k, average, multidim_average, ignore_index)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, multidim_average, ignore_index)
    tp, fp, tn, fn = _multiclass_stat_scores_update(
        preds, target, num_classes, top_k, average, multidim_average, ignore_index, validate_args
    )
    return _stat_reduce(kind, tp, fp, tn, fn, average, multidim_average, beta=beta)


def _multilabel_family(
    kind: str,
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    average: Optional[str] = "macro",
    multidim_average: str = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
    beta: float = 1.0,
) -> Tensor:
    if validate_args:
        if kind == "fbeta":
            _check_beta(beta)
        _multilabel_stat_scores_arg_validation(num_labels, threshold, average, multidim_average, ignore_index)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, multidim_average, ignore_index)
    tp, fp, tn, fn = _multilabel_stat_scores_update(
        preds, target, num_labels, threshold, multidim_average, ignore_index, validate_args
    )
    return _stat_reduce(kind, tp, fp, tn, fn, average, multidim_average, multilabel=True, beta=beta)


def _task_family(
    kind: str,
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
    beta: float = 1.0,
) -> Tensor:
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return _binary_family(kind, preds, target, threshold, multidim_average, ignore_index, validate_args, beta)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        if not isinstance(top_k, int):
            raise ValueError(f"`top_k` is expected to be `int` but `{type(top_k)} was passed.`")
        return _multiclass_family(
            kind, preds, target, num_classes, average, top_k, multidim_average, ignore_index, validate_args, beta
        )
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return _multilabel_family(
            kind, preds, target, num_labels, threshold, average, multidim_average, ignore_index, validate_args, beta
        )
    raise ValueError(f"Unsupported task `{task}` passed.")
