"""Hinge loss (reference ``F/classification/hinge.py:30-289``).

Ignored samples are masked (weight 0) instead of removed with a boolean gather, and the sigmoid/softmax decision is
a device-side select, so an update issues no host synchronisation.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.classification.calibration_error import (
    _binary_float_preds_validation,
    _multiclass_float_preds_validation,
)
from torchmetrics_amd.functional.classification.precision_recall_curve import _prob_or
from torchmetrics_amd.utilities.enums import ClassificationTaskNoMultilabel


def _hinge_loss_compute(measure: Tensor, total: Tensor) -> Tensor:
    return measure / total


def _hinge_on_device(preds: Tensor, target: Tensor, mode: int, squared: bool, ignore_index: Optional[int],
                     size: int) -> Optional[Tensor]:
    """ROCm: the loss in one fused pass (``csrc/classification/hinge.hip``, the kernel the module metrics use) --
    both readings of the scores (as given / sigmoid-or-softmax) accumulated together and the one the batch calls for
    kept on the device, so there is no host round trip.  ``None`` where it does not apply (CPU, gradients to track,
    other dtypes): the ATen formulation below."""
    if not (preds.is_cuda and preds.is_floating_point() and not target.is_floating_point() and preds.numel() > 0
            and preds.dtype in (torch.float32, torch.float16, torch.bfloat16, torch.float64)
            and target.dtype in (torch.int64, torch.int32, torch.uint8, torch.bool)
            and not (torch.is_grad_enabled() and preds.requires_grad)):
        return None
    from torchmetrics_amd import ops
    from torchmetrics_amd.functional.classification.stat_scores import _sink_flag

    acc = torch.float64 if preds.dtype == torch.float64 else torch.float32
    measures = torch.zeros(() if mode != ops.HINGE_ONE_VS_ALL else (size,), dtype=acc, device=preds.device)
    total = torch.zeros((), dtype=torch.int64, device=preds.device)
    if mode == ops.HINGE_BINARY:
        rows = preds.reshape(-1).contiguous()
    else:
        rows = preds.movedim(1, -1).reshape(-1, size).contiguous()
    ops.hinge_update(rows, target.reshape(-1).contiguous(), mode, squared, ignore_index, {}, measures, total,
                     _sink_flag(preds.device))
    return _hinge_loss_compute(measures, total).to(preds.dtype)


def _binary_hinge_loss_arg_validation(squared: bool, ignore_index: Optional[int] = None) -> None:
    if not isinstance(squared, bool):
        raise ValueError(f"Expected argument `squared` to be an bool but got {squared}")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _valid_mask(target: Tensor, ignore_index: Optional[int]) -> Optional[Tensor]:
    return None if ignore_index is None else target != ignore_index


def _binary_hinge_loss_update(
    preds: Tensor, target: Tensor, squared: bool, ignore_index: Optional[int] = None
) -> Tuple[Tensor, Tensor]:
    preds, target = preds.flatten(), target.flatten()
    valid = _valid_mask(target, ignore_index)
    considered = valid
    if preds.numel():
        preds = _prob_or(preds, preds.sigmoid(), considered)
    margin = torch.where(target == 1, preds, -preds)
    measures = torch.clamp(1 - margin, min=0)
    if squared:
        measures = measures.pow(2)
    if valid is not None:
        measures = measures * valid
        total = valid.sum()
    else:
        total = torch.tensor(target.shape[0], device=target.device)
    return measures.sum(dim=0), total


def binary_hinge_loss(
    preds: Tensor,
    target: Tensor,
    squared: bool = False,
    ignore_index: Optional[int] = None,
    validate_args: bool = False,
) -> Tensor:
    """Mean (squared) hinge loss for binary tasks (targets mapped to +-1)."""
    if validate_args:
        _binary_hinge_loss_arg_validation(squared, ignore_index)
        _binary_float_preds_validation(preds, target, ignore_index)
    from torchmetrics_amd import ops

    fused = _hinge_on_device(preds, target, ops.HINGE_BINARY, squared, ignore_index, 1)
    if fused is not None:
        return fused
    measures, total = _binary_hinge_loss_update(preds, target, squared, ignore_index)
    return _hinge_loss_compute(measures, total)


def _multiclass_hinge_loss_arg_validation(
    num_classes: int,
    squared: bool = False,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
) -> None:
    _binary_hinge_loss_arg_validation(squared, ignore_index)
    if not isinstance(num_classes, int) or num_classes < 2:
        raise ValueError(f"Expected argument `num_classes` to be an integer larger than 1, but got {num_classes}")
    allowed_mm = ("crammer-singer", "one-vs-all")
    if multiclass_mode not in allowed_mm:
        raise ValueError(f"Expected argument `multiclass_mode` to be one of {allowed_mm}, but got {multiclass_mode}.")


def _multiclass_hinge_loss_update(
    preds: Tensor,
    target: Tensor,
    squared: bool,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor]:
    c = preds.shape[1]
    preds = preds.movedim(1, -1).reshape(-1, c)
    target = target.flatten()
    valid = _valid_mask(target, ignore_index)
    if preds.numel():
        preds = _prob_or(preds, preds.softmax(1), None if valid is None else valid.unsqueeze(1).expand_as(preds))
    tgt = target.clamp(0, c - 1) if valid is not None else target
    onehot = torch.nn.functional.one_hot(tgt.long(), max(2, c)).bool()[:, :c]
    if multiclass_mode == "crammer-singer":
        own = preds.gather(1, tgt.long().unsqueeze(1)).squeeze(1)
        other = preds.masked_fill(onehot, float("-inf")).max(dim=1).values
        margin = own - other
    else:
        margin = torch.where(onehot, preds, -preds)
    measures = torch.clamp(1 - margin, min=0)
    if squared:
        measures = measures.pow(2)
    if valid is not None:
        measures = measures * (valid if measures.ndim == 1 else valid.unsqueeze(1))
        total = valid.sum()
    else:
        total = torch.tensor(target.shape[0], device=target.device)
    return measures.sum(dim=0), total


def multiclass_hinge_loss(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    squared: bool = False,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
    validate_args: bool = False,
) -> Tensor:
    """Mean (squared) multiclass hinge loss: Crammer-Singer (scalar) or one-vs-all (per class)."""
    if validate_args:
        _multiclass_hinge_loss_arg_validation(num_classes, squared, multiclass_mode, ignore_index)
        _multiclass_float_preds_validation(preds, target, num_classes, ignore_index)
    from torchmetrics_amd import ops

    if preds.ndim >= 2:
        mode = ops.HINGE_CRAMMER_SINGER if multiclass_mode == "crammer-singer" else ops.HINGE_ONE_VS_ALL
        fused = _hinge_on_device(preds, target, mode, squared, ignore_index, preds.shape[1])
        if fused is not None:
            return fused
    measures, total = _multiclass_hinge_loss_update(preds, target, squared, multiclass_mode, ignore_index)
    return _hinge_loss_compute(measures, total)


def hinge_loss(
    preds: Tensor,
    target: Tensor,
    task: Literal["binary", "multiclass"],
    num_classes: Optional[int] = None,
    squared: bool = False,
    multiclass_mode: Literal["crammer-singer", "one-vs-all"] = "crammer-singer",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTaskNoMultilabel.from_str(task)
    if task == ClassificationTaskNoMultilabel.BINARY:
        return binary_hinge_loss(preds, target, squared, ignore_index, validate_args)
    if task == ClassificationTaskNoMultilabel.MULTICLASS:
        if not isinstance(num_classes, int):
            raise ValueError(f"`num_classes` is expected to be `int` but `{type(num_classes)} was passed.`")
        return multiclass_hinge_loss(preds, target, num_classes, squared, multiclass_mode, ignore_index, validate_args)
    raise ValueError(f"Not handled value: {task}")
