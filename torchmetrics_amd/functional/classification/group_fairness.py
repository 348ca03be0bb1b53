"""Group fairness: per-group stat rates, demographic parity, equal opportunity.

Reference: ``F/classification/group_fairness.py:30-382``.  Per-group tp/fp/tn/fn come from one segmented count
(``bincount`` over ``group * 4 + cell``) instead of sorting by group, copying the group sizes to the host and
splitting into Python lists.
"""
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.precision_recall_curve import _prob_or
from torchmetrics_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_tensor_validation,
)
from torchmetrics_amd.utilities.compute import _safe_divide
from torchmetrics_amd.utilities.prints import rank_zero_warn


def _groups_validation(groups: Tensor, num_groups: int) -> None:
    if torch.max(groups) > num_groups:
        raise ValueError(
            f"The largest number in the groups tensor is {torch.max(groups)}, which is larger than the specified",
            f"number of groups {num_groups}. The group identifiers should be ``0, 1, ..., (num_groups - 1)``.",
        )
    if groups.dtype != torch.long:
        raise ValueError(f"Expected dtype of argument groups to be long, not {groups.dtype}.")


def _groups_format(groups: Tensor) -> Tensor:
    return groups.reshape(groups.shape[0], -1)


def _group_stat_counts(
    preds: Tensor, target: Tensor, groups: Tensor, num_groups: int, threshold: float, ignore_index: Optional[int]
) -> Tensor:
    """``[num_groups, 4]`` int64 (tp, fp, tn, fn) per group id, computed on the device in one pass."""
    preds, target = preds.flatten(), target.flatten()
    groups = groups.flatten().long()
    if preds.is_floating_point():
        if preds.numel():
            preds = _prob_or(preds, preds.sigmoid())
        preds = (preds > threshold).long()
    target = target.to(torch.long)
    preds = preds.long()
    valid = torch.ones_like(target, dtype=torch.bool) if ignore_index is None else target != ignore_index
    # cell: 0 tp, 1 fp, 2 tn, 3 fn
    cell = torch.where(preds == 1, torch.where(target == 1, 0, 1), torch.where(target == 0, 2, 3))
    idx = groups * 4 + cell
    counts = torch.zeros(num_groups * 4, dtype=torch.long, device=preds.device)
    counts.index_add_(0, idx.clamp(0, num_groups * 4 - 1), valid.long())
    return counts.view(num_groups, 4)


def _binary_groups_stat_scores(
    preds: Tensor,
    target: Tensor,
    groups: Tensor,
    num_groups: int,
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> List[Tuple[Tensor, Tensor, Tensor, Tensor]]:
    """Stats of the groups present in ``groups`` in ascending id order (reference list contract)."""
    if validate_args:
        _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
        _binary_stat_scores_tensor_validation(preds, target, "global", ignore_index)
        _groups_validation(groups, num_groups)
    # the one host read: which group ids occur (they name the outputs, as the reference's split sizes do)
    present = torch.unique(groups).tolist()
    if not present:
        return []
    G = int(present[-1]) + 1
    if (preds.is_cuda and present[0] >= 0 and target.device == preds.device and groups.device == preds.device
            and preds.numel() == target.numel() == groups.numel()):
        # per-group tp / fp / tn / fn in one pass of the module's kernel (csrc/classification/group_stats.hip)
        tp, fp, tn, fn = (torch.zeros(G, dtype=torch.int64, device=preds.device) for _ in range(4))
        ops.group_stats_update(preds, target, groups, G, threshold, ignore_index, {}, tp, fp, tn, fn)
        counts = torch.stack([tp, fp, tn, fn], 1)
    else:
        lo = min(int(present[0]), 0)
        counts = _group_stat_counts(preds, target, groups - lo, G - lo, threshold, ignore_index)[-lo:] if lo else \
            _group_stat_counts(preds, target, groups, G, threshold, ignore_index)
    return [tuple(counts[g]) for g in present]


def _groups_reduce(group_stats: List[Tuple[Tensor, Tensor, Tensor, Tensor]]) -> Dict[str, Tensor]:
    return {f"group_{g}": torch.stack(s) / torch.stack(s).sum() for g, s in enumerate(group_stats)}


def _groups_stat_transform(group_stats: List[Tuple[Tensor, Tensor, Tensor, Tensor]]) -> Dict[str, Tensor]:
    return {k: torch.stack([s[i] for s in group_stats]) for i, k in enumerate(("tp", "fp", "tn", "fn"))}


def binary_groups_stat_rates(
    preds: Tensor,
    target: Tensor,
    groups: Tensor,
    num_groups: int,
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Dict[str, Tensor]:
    """tp/fp/tn/fn rates of every group present in the batch."""
    group_stats = _binary_groups_stat_scores(preds, target, groups, num_groups, threshold, ignore_index, validate_args)
    return _groups_reduce(group_stats)


def _compute_binary_demographic_parity(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor) -> Dict[str, Tensor]:
    pos_rates = _safe_divide(tp + fp, tp + fp + tn + fn)
    lo, hi = torch.stack([torch.argmin(pos_rates), torch.argmax(pos_rates)]).tolist()  # one read: the key names them
    return {f"DP_{lo}_{hi}": _safe_divide(pos_rates[lo], pos_rates[hi])}


def _compute_binary_equal_opportunity(tp: Tensor, fp: Tensor, tn: Tensor, fn: Tensor) -> Dict[str, Tensor]:
    tpr = _safe_divide(tp, tp + fn)
    lo, hi = torch.stack([torch.argmin(tpr), torch.argmax(tpr)]).tolist()  # one read: the key names them
    return {f"EO_{lo}_{hi}": _safe_divide(tpr[lo], tpr[hi])}


def demographic_parity(
    preds: Tensor, groups: Tensor, threshold: float = 0.5, ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Dict[str, Tensor]:
    """Ratio of the lowest to the highest positive-prediction rate across groups."""
    num_groups = torch.unique(groups).shape[0]
    target = torch.zeros(preds.shape, dtype=torch.long, device=preds.device)
    stats = _binary_groups_stat_scores(preds, target, groups, num_groups, threshold, ignore_index, validate_args)
    return _compute_binary_demographic_parity(**_groups_stat_transform(stats))


def equal_opportunity(
    preds: Tensor, target: Tensor, groups: Tensor, threshold: float = 0.5, ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Dict[str, Tensor]:
    """Ratio of the lowest to the highest true-positive rate across groups."""
    num_groups = torch.unique(groups).shape[0]
    stats = _binary_groups_stat_scores(preds, target, groups, num_groups, threshold, ignore_index, validate_args)
    return _compute_binary_equal_opportunity(**_groups_stat_transform(stats))


def binary_fairness(
    preds: Tensor,
    target: Tensor,
    groups: Tensor,
    task: Literal["demographic_parity", "equal_opportunity", "all"] = "all",
    threshold: float = 0.5,
    ignore_index: Optional[int] = None,
    validate_args: bool = True,
) -> Dict[str, Tensor]:
    if task not in ["demographic_parity", "equal_opportunity", "all"]:
        raise ValueError(
            f"Expected argument `task` to either be ``demographic_parity``,"
            f"``equal_opportunity`` or ``all`` but got {task}."
        )
    if task == "demographic_parity":
        if target is not None:
            rank_zero_warn("The task demographic_parity does not require a target.", UserWarning)
        target = torch.zeros(preds.shape, dtype=torch.long, device=preds.device)
    num_groups = torch.unique(groups).shape[0]
    stats = _groups_stat_transform(
        _binary_groups_stat_scores(preds, target, groups, num_groups, threshold, ignore_index, validate_args)
    )
    if task == "demographic_parity":
        return _compute_binary_demographic_parity(**stats)
    if task == "equal_opportunity":
        return _compute_binary_equal_opportunity(**stats)
    return {**_compute_binary_demographic_parity(**stats), **_compute_binary_equal_opportunity(**stats)}
