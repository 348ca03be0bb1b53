"""Exact match (subset accuracy) for multiclass-multidim and multilabel inputs.

Reference: ``F/classification/exact_match.py:32-258``.
"""
import math
from typing import Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.precision_recall_curve import _prob_or
from torchmetrics_amd.functional.classification.stat_scores import (
    _multiclass_stat_scores_arg_validation,
    _multiclass_stat_scores_tensor_validation,
    _multilabel_stat_scores_arg_validation,
    _multilabel_stat_scores_tensor_validation,
)
from torchmetrics_amd.utilities.compute import _safe_divide
from torchmetrics_amd.utilities.enums import ClassificationTaskNoBinary


def _exact_match_reduce(correct: Tensor, total: Tensor) -> Tensor:
    return _safe_divide(correct, total)


_EM_FLOAT = (torch.float32, torch.float16, torch.bfloat16, torch.float64)


def _exact_match_fused(
    preds: Tensor,
    target: Tensor,
    multilabel: bool,
    num: int,
    threshold: float,
    multidim_average: str,
    ignore_index: Optional[int],
    owner: dict,
    correct: Optional[Tensor] = None,
    total: Optional[Tensor] = None,
) -> Optional[Tuple[Tensor, Tensor]]:
    """ROCm path (``csrc/classification/exact_match.hip``) on the unformatted inputs: argmax / sigmoid-or-not /
    threshold / ignore / all-positions vote in one pass.  Global with ``correct`` / ``total`` given: the states are
    updated in place.  Returns ``(correct, total)`` as the torch update would, or None (the caller's torch body runs)
    for CPU tensors, floating-point targets and shapes the reference's validation rejects (``validate_args=False``
    with mismatched shapes, an argmax over zero classes).  A floating target is compared as-is by the reference
    (``preds == target``: 1.5 matches only 1.5); the kernel compares integer labels, so those batches keep the torch
    body rather than truncating the target.  Every other ROCm input runs here: scores, integer / float label preds,
    ``ignore_index``, empty batches and zero-size position dims (those two in closed form)."""
    if not (preds.is_cuda and target.is_cuda and preds.device == target.device) or target.ndim < 1:
        return None
    if target.is_floating_point():
        return None
    n = target.shape[0]
    samplewise = multidim_average == "samplewise"
    if multilabel:
        if preds.shape != target.shape or preds.ndim < 2:
            return None
        kind, c, p = ops.EM_MULTILABEL, preds.shape[1], math.prod(target.shape[2:])
        total_val = (n * p) if not samplewise else p
    elif preds.ndim == target.ndim + 1:
        if preds.shape[0] != n or preds.shape[2:] != target.shape[1:]:
            return None
        kind, c, p = ops.EM_MULTICLASS, preds.shape[1], math.prod(target.shape[1:])
        total_val = n if not samplewise else 1
    elif preds.ndim == target.ndim:
        if preds.shape[0] != n or preds.numel() != target.numel():
            return None
        # labels (integer target; float preds compare exactly, as `preds == target` does): one unit per sample
        kind, c, p = ops.EM_LABELS, math.prod(target.shape[1:]), 1
        total_val = n if not samplewise else 1
    else:
        return None
    dev = preds.device
    if n == 0 or c == 0 or p == 0:
        if kind == ops.EM_MULTICLASS and c == 0 and n and p:
            return None  # argmax over zero classes: the reference's torch body raises
        # closed form: every vote is over zero positions / labels (vacuously correct) or there are no units
        if kind == ops.EM_MULTILABEL:
            per_sample = p if c == 0 else 0
        else:
            per_sample = 1 if (p == 0 or c == 0) else 0
        if samplewise:
            return (torch.full((n,), per_sample, dtype=torch.int64, device=dev),
                    torch.tensor(total_val, device=dev))
        if correct is None:
            correct = torch.zeros(1, dtype=torch.int64, device=dev)
            total = torch.zeros(1, dtype=torch.int64, device=dev)
        if n * per_sample:
            correct.add_(n * per_sample)
        if total_val:
            total.add_(total_val)
        return correct, total
    preds, target = preds.contiguous(), target.contiguous()
    if target.dtype not in (torch.int64, torch.int32, torch.uint8, torch.bool):
        target = target.long()  # int8 / int16 labels: widened exactly
    if samplewise:
        out = ops.exact_match_update(preds, target, kind, c, p, threshold, ignore_index, True, owner)
        return out, torch.tensor(total_val, device=dev)
    if correct is None:
        correct = torch.zeros(1, dtype=torch.int64, device=dev)
        total = torch.zeros(1, dtype=torch.int64, device=dev)
    ops.exact_match_update(preds, target, kind, c, p, threshold, ignore_index, False, owner, correct, total)
    return correct, total


def _multiclass_exact_match_format(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.ndim == target.ndim + 1:
        preds = preds.argmax(dim=1)
    return preds.reshape(preds.shape[0], -1), target.reshape(target.shape[0], -1)


def _multiclass_exact_match_update(
    preds: Tensor,
    target: Tensor,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
) -> Tuple[Tensor, Tensor]:
    if ignore_index is not None:
        preds = torch.where(target == ignore_index, torch.full_like(preds, ignore_index), preds)
    correct = (preds == target).sum(1) == preds.shape[1]
    correct = correct if multidim_average == "samplewise" else correct.sum()
    total = torch.tensor(preds.shape[0] if multidim_average == "global" else 1, device=correct.device)
    return correct, total


def multiclass_exact_match(
    preds: Tensor,
    target: Tensor,
    num_classes: int,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Fraction of samples whose every position is predicted correctly."""
    if validate_args:
        _multiclass_stat_scores_arg_validation(num_classes, 1, None, multidim_average, ignore_index)
        _multiclass_stat_scores_tensor_validation(preds, target, num_classes, multidim_average, ignore_index)
    fused = _exact_match_fused(preds, target, False, num_classes, 0.5, multidim_average, ignore_index, {})
    if fused is not None:
        correct, total = fused
        return _exact_match_reduce(correct, total) if total.ndim == 0 else _exact_match_reduce(correct[0], total[0])
    preds, target = _multiclass_exact_match_format(preds, target)
    correct, total = _multiclass_exact_match_update(preds, target, multidim_average, ignore_index)
    return _exact_match_reduce(correct, total)


def _multilabel_exact_match_format(
    preds: Tensor, target: Tensor, num_labels: int, threshold: float, ignore_index: Optional[int]
) -> Tuple[Tensor, Tensor]:
    if preds.is_floating_point():
        if preds.numel():
            preds = _prob_or(preds, preds.sigmoid())
        preds = (preds > threshold).long()
    preds = preds.reshape(*preds.shape[:2], -1)
    target = target.reshape(*target.shape[:2], -1)
    if ignore_index is not None:
        # only the target is masked (reference _multilabel_stat_scores_format): an ignored position never matches
        target = target.masked_fill(target == ignore_index, -1)
    return preds, target


def _multilabel_exact_match_update(
    preds: Tensor, target: Tensor, num_labels: int, multidim_average: Literal["global", "samplewise"] = "global"
) -> Tuple[Tensor, Tensor]:
    if multidim_average == "global":
        preds = torch.movedim(preds, 1, -1).reshape(-1, num_labels)
        target = torch.movedim(target, 1, -1).reshape(-1, num_labels)
    correct = ((preds == target).sum(1) == num_labels).sum(dim=-1)
    total = torch.tensor(preds.shape[0 if multidim_average == "global" else 2], device=correct.device)
    return correct, total


def multilabel_exact_match(
    preds: Tensor,
    target: Tensor,
    num_labels: int,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    """Fraction of samples whose whole label set is predicted correctly."""
    if validate_args:
        _multilabel_stat_scores_arg_validation(num_labels, threshold, None, multidim_average, ignore_index)
        _multilabel_stat_scores_tensor_validation(preds, target, num_labels, multidim_average, ignore_index)
    fused = _exact_match_fused(preds, target, True, num_labels, threshold, multidim_average, ignore_index, {})
    if fused is not None:
        correct, total = fused
        return _exact_match_reduce(correct, total) if total.ndim == 0 else _exact_match_reduce(correct[0], total[0])
    preds, target = _multilabel_exact_match_format(preds, target, num_labels, threshold, ignore_index)
    correct, total = _multilabel_exact_match_update(preds, target, num_labels, multidim_average)
    return _exact_match_reduce(correct, total)


def exact_match(
    preds: Tensor,
    target: Tensor,
    task: Literal["multiclass", "multilabel"],
    num_classes: Optional[int] = None,
    num_labels: Optional[int] = None,
    threshold: float = 0.5,
    multidim_average: Literal["global", "samplewise"] = "global",
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Tensor:
    task = ClassificationTaskNoBinary.from_str(task)
    if task == ClassificationTaskNoBinary.MULTICLASS:
        assert num_classes is not None  # noqa: S101
        return multiclass_exact_match(preds, target, num_classes, multidim_average, ignore_index, validate_args)
    if task == ClassificationTaskNoBinary.MULTILABEL:
        assert num_labels is not None  # noqa: S101
        return multilabel_exact_match(preds, target, num_labels, threshold, multidim_average, ignore_index,
                                      validate_args)
    raise ValueError(f"Not handled value: {task}")
