"""Multilabel ranking metrics: coverage error, label ranking average precision, ranking loss.

Reference: ``F/classification/ranking.py:27-267``.  LRAP is computed for all samples at once with sorted rows and a
batched ``searchsorted`` (max-rank tie convention, as the reference's ``_rank_data``) instead of a Python loop with
``torch.unique`` per sample.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops

from torchmetrics_amd.functional.classification.precision_recall_curve import _prob_or
from torchmetrics_amd.utilities.checks import _check_same_shape


def _rank_data(x: Tensor) -> Tensor:
    """Max-rank of every element (1-based count of elements <= it)."""
    _, inverse, counts = torch.unique(x, sorted=True, return_inverse=True, return_counts=True)
    return torch.cumsum(counts, dim=0)[inverse]


def _ranking_reduce(score: Tensor, num_elements) -> Tensor:
    return score / num_elements


def _multilabel_ranking_arg_validation(num_labels: int, ignore_index: Optional[int] = None) -> None:
    if not isinstance(num_labels, int) or num_labels < 2:
        raise ValueError(f"Expected argument `num_labels` to be an integer larger than 1, but got {num_labels}")
    if ignore_index is not None and not isinstance(ignore_index, int):
        raise ValueError(f"Expected argument `ignore_index` to either be `None` or an integer, but got {ignore_index}")


def _multilabel_ranking_tensor_validation(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None
) -> None:
    _check_same_shape(preds, target)
    if preds.shape[1] != num_labels:
        raise ValueError(
            "Expected both `target.shape[1]` and `preds.shape[1]` to be equal to the number of labels"
            f" but got {preds.shape[1]} and expected {num_labels}"
        )
    if target.is_floating_point():
        raise ValueError(f"Expected argument `target` to be an int or long tensor, but got {target.dtype}")
    if not preds.is_floating_point():
        raise ValueError(f"Expected preds tensor to be floating point, but received input with dtype {preds.dtype}")
    uniq = torch.unique(target)
    bad = (uniq != 0) & (uniq != 1)
    if ignore_index is not None:
        bad &= uniq != ignore_index
    if bad.any():
        raise RuntimeError(
            f"Detected the following values in `target`: {uniq} but expected only"
            f" the following values {[0, 1] if ignore_index is None else [0, 1, ignore_index]}."
        )


def _multilabel_ranking_format(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int]
) -> Tuple[Tensor, Tensor]:
    """Sigmoid if logits, ``[N, L, ...] -> [M, L]``, ignored entries mapped to a large negative sentinel."""
    if preds.numel():
        preds = _prob_or(preds, preds.sigmoid())
    preds = preds.movedim(1, -1).reshape(-1, num_labels)
    target = target.movedim(1, -1).reshape(-1, num_labels)
    if ignore_index is not None:
        idx = target == ignore_index
        sentinel = -4 * num_labels
        preds = preds.masked_fill(idx, sentinel)
        target = target.masked_fill(idx, sentinel)
    return preds, target


def _multilabel_coverage_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    fused = ops.label_ranking_rows(preds, target, ops.RANK_COVERAGE)
    if fused is not None:
        return fused[0].sum().to(torch.float32), preds.shape[0]
    offset = torch.where(target == 0, preds.min().abs() + 10, torch.zeros_like(preds))
    preds_min = (preds + offset).min(dim=1)[0]
    coverage = (preds >= preds_min[:, None]).sum(dim=1).to(torch.float32)
    return coverage.sum(), coverage.numel()


def multilabel_coverage_error(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    """How far down the ranked labels one must go to cover all relevant labels (averaged over samples)."""
    if validate_args:
        _multilabel_ranking_arg_validation(num_labels, ignore_index)
        _multilabel_ranking_tensor_validation(preds, target, num_labels, ignore_index)
    preds, target = _multilabel_ranking_format(preds, target, num_labels, ignore_index)
    coverage, total = _multilabel_coverage_error_update(preds, target)
    return _ranking_reduce(coverage, total)


def _multilabel_ranking_average_precision_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    n, num_labels = preds.shape
    if n == 0:
        return torch.tensor(0.0, device=preds.device), 0
    fused = ops.label_ranking_rows(preds, target, ops.RANK_LRAP)
    if fused is not None:
        return fused[0].sum().to(torch.float32), n
    neg = -preds.double()
    relevant = target == 1
    n_rel = relevant.sum(dim=1)
    # max-rank among all labels / among relevant labels (ties count as ranked ahead, as ``_rank_data``)
    all_sorted = neg.sort(dim=1).values
    rank_all = torch.searchsorted(all_sorted, neg, right=True)
    rel_sorted = torch.where(relevant, neg, torch.full_like(neg, float("inf"))).sort(dim=1).values
    rank_rel = torch.searchsorted(rel_sorted, neg, right=True)
    ratio = torch.where(relevant, rank_rel.double() / rank_all.double(), torch.zeros_like(neg))
    per_sample = ratio.sum(dim=1) / n_rel.clamp(min=1)
    degenerate = (n_rel == 0) | (n_rel == num_labels)
    score = torch.where(degenerate, torch.ones_like(per_sample), per_sample).sum().to(torch.float32)
    return score, n


def multilabel_ranking_average_precision(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    """Label ranking average precision (LRAP)."""
    if validate_args:
        _multilabel_ranking_arg_validation(num_labels, ignore_index)
        _multilabel_ranking_tensor_validation(preds, target, num_labels, ignore_index)
    preds, target = _multilabel_ranking_format(preds, target, num_labels, ignore_index)
    score, num_elements = _multilabel_ranking_average_precision_update(preds, target)
    return _ranking_reduce(score, num_elements)


def _multilabel_ranking_loss_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    num_preds, num_labels = preds.shape
    fused = ops.label_ranking_rows(preds, target, ops.RANK_LOSS)
    if fused is not None:
        loss, valid = fused
        total = torch.where(valid.bool().any(), torch.tensor(num_preds, device=preds.device),
                            torch.ones((), device=preds.device, dtype=torch.long))
        return loss.sum().to(torch.float32), total
    relevant = target == 1
    num_relevant = relevant.sum(dim=1)
    valid = (num_relevant > 0) & (num_relevant < num_labels)
    inverse = preds.argsort(dim=1).argsort(dim=1)
    per_label_loss = ((num_labels - inverse) * relevant).to(torch.float32)
    correction = 0.5 * num_relevant * (num_relevant + 1)
    denom = (num_relevant * (num_labels - num_relevant)).clamp(min=1)
    loss = torch.where(valid, (per_label_loss.sum(dim=1) - correction) / denom, torch.zeros_like(correction))
    any_valid = valid.any()
    # reference: when no sample has a mixed label set the update returns (0, 1)
    total = torch.where(any_valid, torch.tensor(num_preds, device=preds.device), torch.ones((), device=preds.device,
                                                                                              dtype=torch.long))
    return loss.sum().to(torch.float32), total


def multilabel_ranking_loss(
    preds: Tensor, target: Tensor, num_labels: int, ignore_index: Optional[int] = None, validate_args: bool = True
) -> Tensor:
    """Average number of incorrectly ordered (relevant, irrelevant) label pairs, normalised per sample."""
    if validate_args:
        _multilabel_ranking_arg_validation(num_labels, ignore_index)
        _multilabel_ranking_tensor_validation(preds, target, num_labels, ignore_index)
    preds, target = _multilabel_ranking_format(preds, target, num_labels, ignore_index)
    loss, num_elements = _multilabel_ranking_loss_update(preds, target)
    return _ranking_reduce(loss, num_elements)
