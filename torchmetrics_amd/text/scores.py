"""Text module metrics (parity: reference ``S/text/*.py``; state names and reductions follow the reference so
state_dicts interchange).  Edit-distance-based metrics run their batched DP on the metric's device (HIP kernel when
the metric lives on a ROCm device)."""
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.text.bleu import (
    _bleu_score_compute,
    _bleu_score_update,
    _SacreBLEUTokenizer,
    _tokenize_fn,
)
from torchmetrics_amd.functional.text.chrf import (
    _N_GRAM_LEVELS,
    _TEXT_LEVELS,
    _chrf_from_stats,
    _chrf_stats,
    _validate_chrf_args,
)
from torchmetrics_amd.functional.text.eed import _check_eed_params, _eed_compute, _eed_update
from torchmetrics_amd.functional.text.error_rates import (
    _cer_update,
    _edit_distance_compute,
    _edit_distance_update,
    _mer_update,
    _wer_update,
    _wip_compute,
    _word_info_lost_compute,
    _word_info_update,
)
from torchmetrics_amd.functional.text.perplexity import _perplexity_compute, _perplexity_update
from torchmetrics_amd.functional.text.rouge import (
    ALLOWED_ACCUMULATE_VALUES,
    ALLOWED_ROUGE_KEYS,
    _normalize_corpus,
    _rouge_score_compute,
    _rouge_score_update,
    _validate_rouge_args,
)
from torchmetrics_amd.functional.text.squad import _squad_compute, _squad_input_check, _squad_update
from torchmetrics_amd.functional.text.ter import _check_ter_flags, _ter_compute, _ter_update, _TercomTokenizer
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat

_Text = Union[str, List[str]]


class _RateMetric(Metric):
    """errors / total style ASR rates (``S/text/{wer,cer,mer}.py``)."""

    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    _update_fn: Callable

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("errors", torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state("total", torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")

    def update(self, preds: _Text, target: _Text) -> None:
        errors, total = type(self)._update_fn(preds, target, self.errors.device)
        self.errors += errors
        self.total += total

    def compute(self) -> Tensor:
        return self.errors / self.total

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class WordErrorRate(_RateMetric):
    """Word error rate (``S/text/wer.py:28``)."""

    _update_fn = staticmethod(_wer_update)


class CharErrorRate(_RateMetric):
    """Character error rate (``S/text/cer.py:28``)."""

    _update_fn = staticmethod(_cer_update)


class MatchErrorRate(_RateMetric):
    """Match error rate (``S/text/mer.py:28``)."""

    _update_fn = staticmethod(_mer_update)


class _WordInfo(Metric):
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("errors", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("target_total", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("preds_total", torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: _Text, target: _Text) -> None:
        errors, tt, pt = _word_info_update(preds, target, self.errors.device)
        self.errors += errors
        self.target_total += tt
        self.preds_total += pt

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class WordInfoLost(_WordInfo):
    """Word information lost (``S/text/wil.py:27``)."""

    higher_is_better: bool = False

    def compute(self) -> Tensor:
        return _word_info_lost_compute(self.errors, self.target_total, self.preds_total)


class WordInfoPreserved(_WordInfo):
    """Word information preserved (``S/text/wip.py:27``; the reference flags it ``higher_is_better=False``)."""

    higher_is_better: bool = False

    def compute(self) -> Tensor:
        return _wip_compute(self.errors, self.target_total, self.preds_total)


class EditDistance(Metric):
    """Character Levenshtein distance (``S/text/edit.py:29``)."""

    higher_is_better: bool = False
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, substitution_cost: int = 1, reduction: Optional[Literal["mean", "sum", "none"]] = "mean",
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not (isinstance(substitution_cost, int) and substitution_cost >= 0):
            raise ValueError(
                f"Expected argument `substitution_cost` to be a positive integer, but got {substitution_cost}"
            )
        self.substitution_cost = substitution_cost
        allowed = (None, "mean", "sum", "none")
        if reduction not in allowed:
            raise ValueError(f"Expected argument `reduction` to be one of {allowed}, but got {reduction}")
        self.reduction = reduction
        if reduction in ("none", None):
            self.add_state("edit_scores_list", default=[], dist_reduce_fx="cat")
        else:
            self.add_state("edit_scores", default=torch.tensor(0), dist_reduce_fx="sum")
            self.add_state("num_elements", default=torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]]) -> None:
        dev = self.edit_scores.device if self.reduction not in ("none", None) else self.device
        distance = _edit_distance_update(preds, target, self.substitution_cost, dev)
        if self.reduction in ("none", None):
            self.edit_scores_list.append(distance)
        else:
            self.edit_scores += distance.sum()
            self.num_elements += distance.shape[0]

    def compute(self) -> Tensor:
        if self.reduction in ("none", None):
            return _edit_distance_compute(dim_zero_cat(self.edit_scores_list), 1, self.reduction)
        return _edit_distance_compute(self.edit_scores, self.num_elements, self.reduction)

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class BLEUScore(Metric):
    """Corpus BLEU (``S/text/bleu.py:33``)."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, n_gram: int = 4, smooth: bool = False, weights: Optional[Sequence[float]] = None,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.n_gram = n_gram
        self.smooth = smooth
        if weights is not None and len(weights) != n_gram:
            raise ValueError(f"List of weights has different weights than `n_gram`: {len(weights)} != {n_gram}")
        self.weights = weights if weights is not None else [1.0 / n_gram] * n_gram
        self.add_state("preds_len", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("target_len", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("numerator", torch.zeros(self.n_gram), dist_reduce_fx="sum")
        self.add_state("denominator", torch.zeros(self.n_gram), dist_reduce_fx="sum")

    def _tokenizer(self) -> Callable[[str], Sequence[str]]:
        return _tokenize_fn

    def update(self, preds: Sequence[str], target: Sequence[Sequence[str]]) -> None:
        self.preds_len, self.target_len = _bleu_score_update(
            preds, target, self.numerator, self.denominator, self.preds_len, self.target_len, self.n_gram,
            self._tokenizer())

    def compute(self) -> Tensor:
        return _bleu_score_compute(self.preds_len, self.target_len, self.numerator, self.denominator, self.n_gram,
                                   self.weights, self.smooth)

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class SacreBLEUScore(BLEUScore):
    """BLEU with SacreBLEU tokenisation (``S/text/sacre_bleu.py:34``)."""

    def __init__(self, n_gram: int = 4, smooth: bool = False, tokenize: str = "13a", lowercase: bool = False,
                 weights: Optional[Sequence[float]] = None, **kwargs: Any) -> None:
        super().__init__(n_gram=n_gram, smooth=smooth, weights=weights, **kwargs)
        self.tokenizer = _SacreBLEUTokenizer(tokenize, lowercase)  # type: ignore[arg-type]

    def _tokenizer(self) -> Callable[[str], Sequence[str]]:
        return self.tokenizer


class CHRFScore(Metric):
    """chrF / chrF++ (``S/text/chrf.py:52``); per-order states named ``total_{preds,target,matching}_{char,word}_{n}_
    grams`` like the reference."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, n_char_order: int = 6, n_word_order: int = 2, beta: float = 2.0, lowercase: bool = False,
                 whitespace: bool = False, return_sentence_level_score: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        _validate_chrf_args(n_char_order, n_word_order, beta)
        self.n_char_order, self.n_word_order, self.beta = n_char_order, n_word_order, beta
        self.lowercase, self.whitespace = lowercase, whitespace
        self.return_sentence_level_score = return_sentence_level_score
        self.n_order = float(n_char_order + n_word_order)
        for name in self._state_names():
            self.add_state(name, torch.tensor(0.0), dist_reduce_fx="sum")
        self.sentence_chrf_score: Optional[List[Tensor]] = None
        if return_sentence_level_score:
            self.add_state("sentence_chrf_score", [], dist_reduce_fx="cat")

    def _state_names(self) -> List[str]:
        """Row-major over (text level in preds/target/matching) x (char orders, word orders)."""
        orders = [("char", n) for n in range(1, self.n_char_order + 1)]
        orders += [("word", n) for n in range(1, self.n_word_order + 1)]
        return [f"total_{text}_{lvl}_{n}_grams" for text in _TEXT_LEVELS for lvl, n in orders]

    def update(self, preds: Sequence[str], target: Sequence[Sequence[str]]) -> None:
        stats, sent = _chrf_stats(preds, target, self.n_char_order, self.n_word_order, self.beta, self.lowercase,
                                  self.whitespace)
        for name, v in zip(self._state_names(), stats.reshape(-1).tolist()):
            setattr(self, name, getattr(self, name) + v)
        if self.return_sentence_level_score:
            self.sentence_chrf_score.append(torch.tensor(sent, dtype=torch.float32, device=self.device))

    def _stats(self) -> Tensor:
        vals = torch.stack([getattr(self, n).double().cpu() for n in self._state_names()])
        return vals.reshape(3, -1)

    def compute(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        score = _chrf_from_stats(self._stats(), self.n_char_order, self.n_word_order, self.beta).to(self.device)
        if self.return_sentence_level_score:
            return score, dim_zero_cat(self.sentence_chrf_score)
        return score

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class TranslationEditRate(Metric):
    """Translation edit rate (``S/text/ter.py:29``)."""

    plot_upper_bound: Optional[float] = 1.0
    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, normalize: bool = False, no_punctuation: bool = False, lowercase: bool = True,
                 asian_support: bool = False, return_sentence_level_score: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        _check_ter_flags(normalize=normalize, no_punctuation=no_punctuation, lowercase=lowercase,
                         asian_support=asian_support)
        self.tokenizer = _TercomTokenizer(normalize, no_punctuation, lowercase, asian_support)
        self.return_sentence_level_score = return_sentence_level_score
        self.add_state("total_num_edits", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total_tgt_len", torch.tensor(0.0), dist_reduce_fx="sum")
        if self.return_sentence_level_score:
            self.add_state("sentence_ter", [], dist_reduce_fx="cat")

    def update(self, preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]]) -> None:
        self.total_num_edits, self.total_tgt_len, sent = _ter_update(
            preds, target, self.tokenizer, self.total_num_edits, self.total_tgt_len,
            [] if self.return_sentence_level_score else None)
        if self.return_sentence_level_score:
            self.sentence_ter.extend(s.to(self.device) for s in sent)

    def compute(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        ter = _ter_compute(self.total_num_edits, self.total_tgt_len)
        if self.return_sentence_level_score:
            return ter, dim_zero_cat(self.sentence_ter)
        return ter

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class ExtendedEditDistance(Metric):
    """Extended edit distance (``S/text/eed.py:28``)."""

    # compute() averages the per-update sentence-score tensors element by element: keep the list structure
    _fold_cat_lists = False
    higher_is_better: bool = False
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, language: Literal["en", "ja"] = "en", return_sentence_level_score: bool = False,
                 alpha: float = 2.0, rho: float = 0.3, deletion: float = 0.2, insertion: float = 1.0,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if language not in ("en", "ja"):
            raise ValueError(f"Expected argument `language` to either be `en` or `ja` but got {language}")
        self.language = language
        self.return_sentence_level_score = return_sentence_level_score
        _check_eed_params(alpha, rho, deletion, insertion)
        self.alpha, self.rho, self.deletion, self.insertion = alpha, rho, deletion, insertion
        self.add_state("sentence_eed", [], dist_reduce_fx="cat")

    def update(self, preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]]) -> None:
        scores = _eed_update(preds, target, self.language, self.alpha, self.rho, self.deletion, self.insertion)
        self.sentence_eed.extend(s.to(self.device) for s in scores)

    def compute(self) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        avg = _eed_compute(self.sentence_eed)
        if self.return_sentence_level_score:
            return avg, dim_zero_cat(self.sentence_eed)
        return avg

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class ROUGEScore(Metric):
    """ROUGE-N / L / Lsum (``S/text/rouge.py:36``); list states ``rouge<key>_{fmeasure,precision,recall}``."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, use_stemmer: bool = False, normalizer: Optional[Callable[[str], str]] = None,
                 tokenizer: Optional[Callable[[str], Sequence[str]]] = None,
                 accumulate: Literal["avg", "best"] = "best",
                 rouge_keys: Union[str, Tuple[str, ...]] = ("rouge1", "rouge2", "rougeL", "rougeLsum"),
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rouge_keys, self.stemmer = _validate_rouge_args(use_stemmer, rouge_keys)
        if accumulate not in ALLOWED_ACCUMULATE_VALUES:
            raise ValueError(
                f"Got unknown accumulate value {accumulate}. Expected to be one of {ALLOWED_ACCUMULATE_VALUES}"
            )
        self.rouge_keys = rouge_keys
        self.rouge_keys_values = [ALLOWED_ROUGE_KEYS[k] for k in rouge_keys]
        self.normalizer, self.tokenizer, self.accumulate = normalizer, tokenizer, accumulate
        for key in self.rouge_keys:
            for score in ("fmeasure", "precision", "recall"):
                self.add_state(f"{key}_{score}", [], dist_reduce_fx=None)

    def update(self, preds: Union[str, Sequence[str]],
               target: Union[str, Sequence[str], Sequence[Sequence[str]]]) -> None:
        preds, target = _normalize_corpus(preds, target)
        out = _rouge_score_update(preds, target, self.rouge_keys_values, self.accumulate, self.stemmer,
                                  self.normalizer, self.tokenizer)
        for key, lst in out.items():
            for d in lst:
                for tp, v in d.items():
                    getattr(self, f"rouge{key}_{tp}").append(v.to(self.device))

    def compute(self) -> Dict[str, Tensor]:
        out = {}
        for key in self.rouge_keys_values:
            for tp in ("fmeasure", "precision", "recall"):
                out[f"rouge{key}_{tp}"] = getattr(self, f"rouge{key}_{tp}")
        return _rouge_score_compute(out)

    def __hash__(self) -> int:
        vals = [self.__class__.__name__]
        for key in self._defaults:
            v = getattr(self, key)
            vals.append(tuple(v) if isinstance(v, list) else v)
        return hash(tuple(vals))

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class SQuAD(Metric):
    """SQuAD exact match / F1 (``S/text/squad.py:34``)."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 100.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state(name="f1_score", default=torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state(name="exact_match", default=torch.tensor(0, dtype=torch.float), dist_reduce_fx="sum")
        self.add_state(name="total", default=torch.tensor(0, dtype=torch.int), dist_reduce_fx="sum")

    def update(self, preds: Any, target: Any) -> None:
        preds_dict, target_dict = _squad_input_check(preds, target)
        f1, em, total = _squad_update(preds_dict, target_dict)
        self.f1_score += f1.to(self.f1_score)
        self.exact_match += em.to(self.exact_match)
        self.total += total.to(self.total)

    def compute(self) -> Dict[str, Tensor]:
        return _squad_compute(self.f1_score, self.exact_match, self.total)

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class Perplexity(Metric):
    """Perplexity over ``[B, S, V]`` logits (``S/text/perplexity.py:28``) on the fused token-NLL kernel."""

    is_differentiable = True
    higher_is_better = False
    full_state_update = False

    def __init__(self, ignore_index: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if ignore_index is not None and not isinstance(ignore_index, int):
            raise ValueError(f"Argument `ignore_index` expected to either be `None` or an `int` but got {ignore_index}")
        self.ignore_index = ignore_index
        self.add_state("total_log_probs", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("count", default=torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        flag = self._device_error_buffer(preds.device) if preds.is_cuda else None
        total, count = _perplexity_update(preds, target, self.ignore_index, flag)
        self.total_log_probs = self.total_log_probs + total.to(self.total_log_probs.dtype)
        self.count = self.count + count

    def compute(self) -> Tensor:
        self._raise_device_errors()
        return _perplexity_compute(self.total_log_probs, self.count)

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


__all__ = [
    "BLEUScore", "CharErrorRate", "CHRFScore", "EditDistance", "ExtendedEditDistance", "MatchErrorRate",
    "Perplexity", "ROUGEScore", "SacreBLEUScore", "SQuAD", "TranslationEditRate", "WordErrorRate", "WordInfoLost",
    "WordInfoPreserved",
]
