"""chrF / chrF++ (reference ``F/text/chrf.py``).

Per sentence the character n-grams are substrings of the (optionally whitespace-stripped) sentence and the word
n-grams tuples of punctuation-split words, counted with ``collections.Counter``; clipped matches are the size of the
multiset intersection.  Statistics are kept as three ``[n_char + n_word]`` float64 vectors (hypothesis totals,
best-reference totals, matches) and the F-beta is evaluated vectorised, instead of the reference's per-count tensor
dictionaries.
"""
from collections import Counter
from itertools import chain
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd.functional.text.helper import _validate_inputs

_EPS_SMOOTHING = 1e-16
_PUNCTUATIONS = set("!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~")
_N_GRAM_LEVELS = ("char", "word")
_TEXT_LEVELS = ("preds", "target", "matching")


def _get_characters(sentence: str, whitespace: bool) -> str:
    return sentence if whitespace else sentence.strip().replace(" ", "")


def _separate_word_and_punctuation(word: str) -> List[str]:
    if len(word) == 1:
        return [word]
    if word[-1] in _PUNCTUATIONS:
        return [word[:-1], word[-1]]
    if word[0] in _PUNCTUATIONS:
        return [word[0], word[1:]]
    return [word]


def _get_words_and_punctuation(sentence: str) -> List[str]:
    return list(chain.from_iterable(_separate_word_and_punctuation(w) for w in sentence.strip().split()))


def _sentence_counters(sentence: str, n_char: int, n_word: int, lowercase: bool,
                       whitespace: bool) -> List[Counter]:
    """One Counter per order: char orders 1..n_char then word orders 1..n_word."""
    if lowercase:
        sentence = sentence.lower()
    chars = _get_characters(sentence, whitespace)
    words = _get_words_and_punctuation(sentence)
    out = [Counter(chars[i:i + n] for i in range(len(chars) - n + 1)) for n in range(1, n_char + 1)]
    out += [Counter(tuple(words[i:i + n]) for i in range(len(words) - n + 1)) for n in range(1, n_word + 1)]
    return out


def _totals(counters: List[Counter]) -> np.ndarray:
    return np.array([sum(c.values()) for c in counters], dtype=np.float64)


def _fscore(match: np.ndarray, hyp: np.ndarray, ref: np.ndarray, n_order: float, beta: float) -> float:
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(hyp > 0, match / np.where(hyp > 0, hyp, 1), 0.0)
        rec = np.where(ref > 0, match / np.where(ref > 0, ref, 1), 0.0)
    den = np.maximum(beta**2 * prec + rec, _EPS_SMOOTHING)
    return float(((1 + beta**2) * prec * rec / den).sum() / n_order)


def _chrf_stats(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]], n_char: int,
                n_word: int, beta: float, lowercase: bool, whitespace: bool) -> Tuple[np.ndarray, List[float]]:
    """``stats [3, n_char + n_word]`` = (hypothesis, best-reference, matching) totals and sentence scores."""
    target_corpus, preds = _validate_inputs(target, preds)
    n_order = float(n_char + n_word)
    stats = np.zeros((3, n_char + n_word), dtype=np.float64)
    sentence_scores: List[float] = []
    for pred, refs in zip(preds, target_corpus):
        pc = _sentence_counters(pred, n_char, n_word, lowercase, whitespace)
        hyp_tot = _totals(pc)
        stats[0] += hyp_tot
        best, best_ref, best_match = 0.0, np.zeros_like(hyp_tot), np.zeros_like(hyp_tot)
        for ref in refs:
            rc = _sentence_counters(ref, n_char, n_word, lowercase, whitespace)
            match = np.array([sum((a & b).values()) for a, b in zip(pc, rc)], dtype=np.float64)
            ref_tot = _totals(rc)
            f = _fscore(match, hyp_tot, ref_tot, n_order, beta)
            if f > best:  # first strictly-better reference; none > 0 leaves zero target/matching stats
                best, best_ref, best_match = f, ref_tot, match
        stats[1] += best_ref
        stats[2] += best_match
        sentence_scores.append(best)
    return stats, sentence_scores


def _chrf_from_stats(stats: Union[np.ndarray, Tensor], n_char: int, n_word: int, beta: float) -> Tensor:
    s = stats.detach().cpu().double().numpy() if isinstance(stats, Tensor) else stats
    return torch.tensor(_fscore(s[2], s[0], s[1], float(n_char + n_word), beta), dtype=torch.float32)


def _validate_chrf_args(n_char_order: int, n_word_order: int, beta: float) -> None:
    if not isinstance(n_char_order, int) or n_char_order < 1:
        raise ValueError("Expected argument `n_char_order` to be an integer greater than or equal to 1.")
    if not isinstance(n_word_order, int) or n_word_order < 0:
        raise ValueError("Expected argument `n_word_order` to be an integer greater than or equal to 0.")
    if beta < 0:
        raise ValueError("Expected argument `beta` to be greater than 0.")


def chrf_score(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]], n_char_order: int = 6,
               n_word_order: int = 2, beta: float = 2.0, lowercase: bool = False, whitespace: bool = False,
               return_sentence_level_score: bool = False) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """Corpus chrF (``n_word_order=0``) / chrF++ (default) score (``F/text/chrf.py``)."""
    _validate_chrf_args(n_char_order, n_word_order, beta)
    stats, sent = _chrf_stats(preds, target, n_char_order, n_word_order, beta, lowercase, whitespace)
    score = _chrf_from_stats(stats, n_char_order, n_word_order, beta)
    if return_sentence_level_score:
        return score, torch.tensor(sent, dtype=torch.float32)
    return score
