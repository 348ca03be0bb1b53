"""Confusion matrices (functional). Parity: reference ``F/classification/confusion_matrix.py:26-665``.

Binary ``[2, 2]``, multiclass ``[C, C]`` and multilabel ``[L, 2, 2]`` matrices (rows = target, cols = prediction)
are accumulated *in place* by the fused HIP kernels of ``csrc/classification/stat_scores.hip``:

* multiclass: one wave64 per row computes the argmax of ``[N, C]`` scores with 16-byte vector loads and does a single
  64-bit atomic increment of ``confmat[target, argmax]`` (LDS-privatised when ``C*C`` is small);
* binary / multilabel: threshold (+ sigmoid auto-detection without a host sync) and per-label counters.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.stat_scores import (
    _as_preds,
    _as_target,
    _binary_stat_scores_tensor_validation,
    _check_flag,
    _Ctx,
    _multiclass_stat_scores_tensor_validation,
    _multilabel_stat_scores_tensor_validation,
    _scratch_flag,
    _sink_flag,
)
from torchmetrics_amd.utilities.enums import ClassificationTask
from torchmetrics_amd.utilities.prints import rank_zero_warn

_ALLOWED_NORMALIZE = ("true", "pred", "all", "none", None)


def _confusion_matrix_reduce(confmat: Tensor, normalize: Optional[str] = None) -> Tensor:
    """Normalise over true labels (rows), predictions (cols) or everything; NaNs from empty rows become 0."""
    if normalize not in _ALLOWED_NORMALIZE:
        raise ValueError(f"Argument `normalize` needs to one of the following: {_ALLOWED_NORMALIZE}")
    if normalize is None or normalize == "none":
        return confmat
    cm = confmat if confmat.is_floating_point() else confmat.float()
    dims = {"true": [-1], "pred": [-2], "all": [-2, -1]}[normalize]
    cm = cm / cm.sum(dim=dims, keepdim=True)
    nans = torch.isnan(cm)
    n_nan = int(nans.sum())
    if n_nan:
        cm = torch.where(nans, torch.zeros_like(cm), cm)
        rank_zero_warn(f"{n_nan} NaN values found in confusion matrix have been replaced with zeros.")
    return cm


# ------------------------------------------------------------------------------------------------------ validation
def _binary_confusion_matrix_arg_validation(
    threshold: float = 0.5, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float in the [0,1] range, but got {threshold}.")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")
    if normalize not in _ALLOWED_NORMALIZE:
        raise ValueError(f"Expected argument `normalize` to be one of {_ALLOWED_NORMALIZE}, but got {normalize}.")


def _binary_confusion_matrix_tensor_validation(preds: Tensor, target: Tensor, ignore_index: Optional[int] = None) -> None:
    _binary_stat_scores_tensor_validation(preds, target, "global", ignore_index)


def _multiclass_confusion_matrix_arg_validation(
    num_classes: int, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")
    if normalize not in _ALLOWED_NORMALIZE:
        raise ValueError(f"Expected argument `normalize` to be one of {_ALLOWED_NORMALIZE}, but got {normalize}.")


def _multiclass_confusion_matrix_tensor_validation(
    preds: Tensor, target: Tensor, num_classes: int, ignore_index: Optional[int] = None
) -> None:
    _multiclass_stat_scores_tensor_validation(preds, target, num_classes, "global", ignore_index)


def _multilabel_confusion_matrix_arg_validation(
    num_labels: int, threshold: float = 0.5, ignore_index: Optional[int] = None, normalize: Optional[str] = None
) -> None:
    if not isinstance(num_labels, int) or num_labels < 2:
        raise ValueError(f"Expected argument `num_labels` to be an integer larger than 1, but got {num_labels}")
    if not (isinstance(threshold, float) and (0 <= threshold <= 1)):
        raise ValueError(f"Expected argument `threshold` to be a float, but got {threshold}.")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")
    if normalize not in _ALLOWED_NORMALIZE:
        raise ValueError(f"Expected argument `normalize` to be one of {_ALLOWED_NORMALIZE}, but got {normalize}.")


def _multilabel_confusion_matrix_tensor_validation(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None
) -> None:
    _multilabel_stat_scores_tensor_validation(preds, target, num_labels, "global", ignore_index)


# ------------------------------------------------------------------------------------------------ fused updates
def _binary_confmat_accumulate(
    preds: Tensor, target: Tensor, confmat: Tensor, threshold: float, ignore_index: Optional[int],
    flag: Optional[Tensor], workspace: Optional[Tuple[Tensor, Tensor]] = None,
) -> None:
    """``confmat[2,2] += batch`` (ignored positions excluded from the logit auto-detection, as the reference)."""
    p, t = _as_preds(preds).reshape(-1), _as_target(target).reshape(-1)
    ws, not_prob = workspace if workspace is not None else (
        torch.zeros(7, dtype=torch.int64, device=p.device), torch.zeros(1, dtype=torch.int32, device=p.device))
    flag = flag if flag is not None else _sink_flag(p.device)
    ops.bin_update(p, t, ws, flag, not_prob, 1, threshold, ignore_index, False, prob_check_all=False)
    ops.bin_confmat_finalize(ws, not_prob, confmat)


def _multilabel_confmat_accumulate(
    preds: Tensor, target: Tensor, confmat: Tensor, num_labels: int, threshold: float, ignore_index: Optional[int],
    flag: Optional[Tensor], workspace: Optional[Tuple[Tensor, Tensor]] = None,
) -> None:
    p, t = _as_preds(preds), _as_target(target)
    ws, not_prob = workspace if workspace is not None else (
        torch.zeros(7 * num_labels, dtype=torch.int64, device=p.device),
        torch.zeros(1, dtype=torch.int32, device=p.device))
    flag = flag if flag is not None else _sink_flag(p.device)
    ops.bin_update(p, t, ws, flag, not_prob, num_labels, threshold, ignore_index, False, prob_check_all=True)
    ops.bin_confmat_finalize(ws, not_prob, confmat)


def _multiclass_confmat_accumulate(
    preds: Tensor, target: Tensor, confmat: Tensor, num_classes: int, ignore_index: Optional[int],
    flag: Optional[Tensor],
) -> None:
    t = _as_target(target)
    p = preds if preds.is_floating_point() and preds.ndim == t.ndim + 1 else _as_preds(preds)
    if t.ndim == 0:
        t, p = t.reshape(1), p.reshape(1, *p.shape) if p.ndim == 1 else p.reshape(1)
    flag = flag if flag is not None else _sink_flag(p.device)
    ops.mc_update(p, t, confmat, flag, num_classes, ignore_index, ops.MC_CONFMAT, False)


# ---------------------------------------------------------------------------------------------------- public API
def binary_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    threshold: float = 0.5,
    normalize: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[2, 2]`` confusion matrix for binary tasks."""
    if validate_args:
        _binary_confusion_matrix_arg_validation(threshold, ignore_index, normalize)
        _binary_confusion_matrix_tensor_validation(preds, target, ignore_index)
    confmat = torch.zeros(2, 2, dtype=torch.long, device=preds.device)
    flag = _scratch_flag(preds.device)
    _binary_confmat_accumulate(preds, target, confmat, threshold, ignore_index, flag)
    if validate_args:
        _check_flag(flag)
    return _confusion_matrix_reduce(confmat, normalize)


def multiclass_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    normalize: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[C, C]`` confusion matrix for multiclass tasks (scores are arg-maxed over dim 1)."""
    if validate_args:
        _multiclass_confusion_matrix_arg_validation(num_classes, ignore_index, normalize)
        _multiclass_confusion_matrix_tensor_validation(preds, target, num_classes, ignore_index)
    confmat = torch.zeros(num_classes, num_classes, dtype=torch.long, device=preds.device)
    flag = _scratch_flag(preds.device)
    _multiclass_confmat_accumulate(preds, target, confmat, num_classes, ignore_index, flag)
    if validate_args:
        _check_flag(flag, _Ctx(num_classes=num_classes))
    return _confusion_matrix_reduce(confmat, normalize)


def multilabel_confusion_matrix(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    normalize: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """``[L, 2, 2]`` confusion matrices for multilabel tasks."""
    if validate_args:
        _multilabel_confusion_matrix_arg_validation(num_labels, threshold, ignore_index, normalize)
        _multilabel_confusion_matrix_tensor_validation(preds, target, num_labels, ignore_index)
    confmat = torch.zeros(num_labels, 2, 2, dtype=torch.long, device=preds.device)
    flag = _scratch_flag(preds.device)
    _multilabel_confmat_accumulate(preds, target, confmat, num_labels, threshold, ignore_index, flag)
    if validate_args:
        _check_flag(flag)
    return _confusion_matrix_reduce(confmat, normalize)


def confusion_matrix(
    preds: Tensor,
    target: Tensor,
    task: str,
    threshold: float = 0.5,
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    normalize: Optional[str] = None,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Task-dispatching confusion matrix."""
    task = ClassificationTask.from_str(task)
    if task == ClassificationTask.BINARY:
        return binary_confusion_matrix(preds, target, threshold, normalize, ignore_index, validate_args)
    if task == ClassificationTask.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_confusion_matrix(preds, target, num_classes, normalize, ignore_index, validate_args)
    if task == ClassificationTask.MULTILABEL:
        if not isinstance(num_labels, int):
            raise ValueError(f"`num_labels` is expected to be `int` but `{type(num_labels)} was passed.`")
        return multilabel_confusion_matrix(preds, target, num_labels, threshold, normalize, ignore_index, validate_args)
    raise ValueError(f"Task {task} not supported.")
