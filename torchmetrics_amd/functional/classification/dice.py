"""Dice score with the legacy (task-less) input API (reference ``F/classification/dice.py:24-160``).

Dice is the F1 of the legacy stat scores: ``2 tp / (2 tp + fp + fn)``.  Both terms come from one stack of the
counts; classes that never occur are dropped (macro) or marked with a ``-1`` sentinel that the shared legacy reducer
turns into NaN (``average=None``).
"""
from typing import Optional

import torch
from torch import Tensor

from torchmetrics_amd.functional.classification._legacy import (
    _input_squeeze,
    _reduce_stat_scores,
    _stat_scores_update,
)
from torchmetrics_amd.utilities.enums import AverageMethod, MDMCAverageMethod

_AVERAGES = ("micro", "macro", "weighted", "samples", "none", None)
_PER_CLASS = ("macro", "weighted", "none", None)
_MDMC = [None, "samplewise", "global"]


def _dice_compute(
    tp: Tensor,
    fp: Tensor,
    fn: Tensor,
    average: Optional[str],
    mdmc_average: Optional[str],
    zero_division: int = 0,
) -> Tensor:
    terms = torch.stack([2 * tp, 2 * tp + fp + fn])  # [numerator, denominator]
    if mdmc_average != MDMCAverageMethod.SAMPLEWISE:
        absent = (tp + fp + fn) == 0
        if average == AverageMethod.MACRO:
            terms = terms[:, ~absent]
        elif average == AverageMethod.NONE:
            terms = terms.masked_fill(absent.unsqueeze(0), -1)
    return _reduce_stat_scores(
        numerator=terms[0],
        denominator=terms[1],
        weights=tp + fn if average == "weighted" else None,
        average=average,
        mdmc_average=mdmc_average,
        zero_division=zero_division,
    )


def _check_dice_args(average: Optional[str], mdmc_average: Optional[str], num_classes: Optional[int],
                     ignore_index: Optional[int], top_k: Optional[int]) -> None:
    if average not in _AVERAGES:
        raise ValueError(f"The `average` has to be one of {_AVERAGES}, got {average}.")
    if average in _PER_CLASS and (not num_classes or num_classes < 1):
        raise ValueError(f"When you set `average` as {average}, you have to provide the number of classes.")
    if mdmc_average not in _MDMC:
        raise ValueError(f"The `mdmc_average` has to be one of {_MDMC}, got {mdmc_average}.")
    bad_ignore = num_classes and ignore_index is not None and (ignore_index >= num_classes or num_classes == 1)
    if bad_ignore:
        raise ValueError(f"The `ignore_index` {ignore_index} is not valid for inputs with {num_classes} classes")
    if top_k is not None and not (isinstance(top_k, int) and top_k > 0):
        raise ValueError(f"The `top_k` should be an integer larger than 0, got {top_k}")


def dice(
    preds: Tensor,
    target: Tensor,
    zero_division: int = 0,
    average: Optional[str] = "micro",
    mdmc_average: Optional[str] = "global",
    threshold: float = 0.5,
    top_k: Optional[int] = None,
    num_classes: Optional[int] = None,
    multiclass: Optional[bool] = None,
    ignore_index: Optional[int] = None,
) -> Tensor:
    """Dice coefficient ``2 tp / (2 tp + fp + fn)`` with micro / macro / weighted / samples / none averaging."""
    _check_dice_args(average, mdmc_average, num_classes, ignore_index, top_k)
    preds, target = _input_squeeze(preds, target)
    tp, fp, _, fn = _stat_scores_update(
        preds, target, reduce="macro" if average in ("weighted", "none", None) else average,
        mdmc_reduce=mdmc_average, threshold=threshold, num_classes=num_classes, top_k=top_k, multiclass=multiclass,
        ignore_index=ignore_index,
    )
    return _dice_compute(tp, fp, fn, average, mdmc_average, zero_division)
