"""ASR error rates and Levenshtein edit distance (reference ``F/text/{wer,cer,mer,wil,wip,edit}.py``).

All five rates reduce to per-pair edit distances plus token counts; one batched edit-distance call
(:func:`torchmetrics_amd.functional.text._edit.batched_edit_distance`) serves the whole batch, and the sums are
taken on the device that will hold the metric state.
"""
from typing import List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.text._edit import _as_list, batched_edit_distance, tokenize_pairs

_Text = Union[str, List[str]]


def _pair_stats(preds: _Text, target: _Text, level: str = "word",
                device: Optional[torch.device] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """(edit distances [B] float, pred lengths [B], target lengths [B])."""
    preds, target = _as_list(preds), _as_list(target)
    n = min(len(preds), len(target))  # the reference zips
    p_ids, t_ids = tokenize_pairs(preds[:n], target[:n], level)
    dist = batched_edit_distance(p_ids, t_ids, device=device).to(torch.float32)
    plen = torch.tensor([len(x) for x in p_ids], dtype=torch.float32, device=dist.device)
    tlen = torch.tensor([len(x) for x in t_ids], dtype=torch.float32, device=dist.device)
    return dist, plen, tlen


def _wer_update(preds: _Text, target: _Text, device: Optional[torch.device] = None) -> Tuple[Tensor, Tensor]:
    dist, _, tlen = _pair_stats(preds, target, "word", device)
    return dist.sum(), tlen.sum()


def _wer_compute(errors: Tensor, total: Tensor) -> Tensor:
    return errors / total


def word_error_rate(preds: _Text, target: _Text) -> Tensor:
    """Word error rate: word-level edit operations per reference word (``F/text/wer.py``)."""
    return _wer_compute(*_wer_update(preds, target))


def _cer_update(preds: _Text, target: _Text, device: Optional[torch.device] = None) -> Tuple[Tensor, Tensor]:
    dist, _, tlen = _pair_stats(preds, target, "char", device)
    return dist.sum(), tlen.sum()


_cer_compute = _wer_compute


def char_error_rate(preds: _Text, target: _Text) -> Tensor:
    """Character error rate: character-level edit operations per reference character (``F/text/cer.py``)."""
    return _cer_compute(*_cer_update(preds, target))


def _mer_update(preds: _Text, target: _Text, device: Optional[torch.device] = None) -> Tuple[Tensor, Tensor]:
    dist, plen, tlen = _pair_stats(preds, target, "word", device)
    return dist.sum(), torch.maximum(plen, tlen).sum()


_mer_compute = _wer_compute


def match_error_rate(preds: _Text, target: _Text) -> Tensor:
    """Match error rate: edits per max(|pred|, |target|) word (``F/text/mer.py``)."""
    return _mer_compute(*_mer_update(preds, target))


def _word_info_update(preds: _Text, target: _Text,
                      device: Optional[torch.device] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """(``errors - total`` = minus the number of hits, target words, pred words) as in ``F/text/wil.py``."""
    dist, plen, tlen = _pair_stats(preds, target, "word", device)
    return dist.sum() - torch.maximum(plen, tlen).sum(), tlen.sum(), plen.sum()


_word_info_lost_update = _wip_update = _word_info_update


def _wip_compute(errors: Tensor, target_total: Tensor, preds_total: Tensor) -> Tensor:
    return (errors / target_total) * (errors / preds_total)


def _word_info_lost_compute(errors: Tensor, target_total: Tensor, preds_total: Tensor) -> Tensor:
    return 1 - _wip_compute(errors, target_total, preds_total)


def word_information_preserved(preds: _Text, target: _Text) -> Tensor:
    """Word information preserved: hits^2 / (|target| |pred|) (``F/text/wip.py``)."""
    return _wip_compute(*_wip_update(preds, target))


def word_information_lost(preds: _Text, target: _Text) -> Tensor:
    """Word information lost: 1 - WIP (``F/text/wil.py``)."""
    return _word_info_lost_compute(*_word_info_lost_update(preds, target))


def _edit_distance_update(preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]],
                          substitution_cost: int = 1, device: Optional[torch.device] = None) -> Tensor:
    preds, target = _as_list(preds), _as_list(target)
    if not all(isinstance(x, str) for x in preds):
        raise ValueError(f"Expected all values in argument `preds` to be string type, but got {preds}")
    if not all(isinstance(x, str) for x in target):
        raise ValueError(f"Expected all values in argument `target` to be string type, but got {target}")
    if len(preds) != len(target):
        raise ValueError(
            f"Expected argument `preds` and `target` to have same length, but got {len(preds)} and {len(target)}"
        )
    p_ids, t_ids = tokenize_pairs(preds, target, "char")
    # tercom-style beam-limited DP, like the reference's `_LevenshteinEditDistance` (F/text/edit.py:44)
    return batched_edit_distance(p_ids, t_ids, substitution_cost, beam=True, device=device).to(torch.int32)


def _edit_distance_compute(edit_scores: Tensor, num_elements: Union[Tensor, int],
                           reduction: Optional[Literal["mean", "sum", "none"]] = "mean") -> Tensor:
    if edit_scores.numel() == 0:
        return torch.tensor(0, dtype=torch.int32)
    if reduction == "mean":
        return edit_scores.sum() / num_elements
    if reduction == "sum":
        return edit_scores.sum()
    if reduction is None or reduction == "none":
        return edit_scores
    raise ValueError("Expected argument `reduction` to either be 'sum', 'mean', 'none' or None")


def edit_distance(preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]], substitution_cost: int = 1,
                  reduction: Optional[Literal["mean", "sum", "none"]] = "mean") -> Tensor:
    """Character Levenshtein distance between paired strings (``F/text/edit.py:78``)."""
    distance = _edit_distance_update(preds, target, substitution_cost)
    return _edit_distance_compute(distance, distance.numel(), reduction)
