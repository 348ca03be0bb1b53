"""BLEU and SacreBLEU (reference ``F/text/bleu.py``, ``F/text/sacre_bleu.py``).

Tokenisation is host-side string work; the n-gram clipping runs vectorised over the whole batch
(:mod:`torchmetrics_amd.functional.text._ngram`) and only the four ``[n_gram]`` sums are added to the (device)
state.
"""
import importlib.util
import os
import re
import tempfile
from functools import lru_cache
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd.functional.text._ngram import clipped_ngram_counts, ids_of

_TokenizersLiteral = Literal["none", "13a", "zh", "intl", "char", "ja-mecab", "ko-mecab", "flores101", "flores200"]
AVAILABLE_TOKENIZERS = ("none", "13a", "zh", "intl", "char", "ja-mecab", "ko-mecab", "flores101", "flores200")
_FLORES_LOCAL_DIR = os.path.join(tempfile.gettempdir(), "torchmetrics-flores")
_FLORES_FILES = {"flores101": "sacrebleu_tokenizer_spm.model", "flores200": "flores200_sacrebleu_tokenizer_spm.model"}


def _tokenize_fn(sentence: str) -> Sequence[str]:
    return sentence.split()


def _bleu_score_update(preds: Sequence[str], target: Sequence[Sequence[str]], numerator: Tensor, denominator: Tensor,
                       preds_len: Tensor, target_len: Tensor, n_gram: int = 4,
                       tokenizer: Callable[[str], Sequence[str]] = _tokenize_fn) -> Tuple[Tensor, Tensor]:
    """Accumulate clipped n-gram matches / totals into ``numerator`` / ``denominator`` in place and return the updated
    (prediction length, closest-reference length) sums."""
    vocab: Dict[str, int] = {}
    p_ids: List[np.ndarray] = []
    r_ids: List[List[np.ndarray]] = []
    plen = tlen = 0
    for pred, tgts in zip(preds, target):
        pt = ids_of(tokenizer(pred) if pred else [], vocab)
        rts = [ids_of(tokenizer(t) if t else [], vocab) for t in tgts]
        p_ids.append(pt)
        r_ids.append(rts)
        plen += len(pt)
        lens = [len(r) for r in rts]
        diffs = [abs(len(pt) - x) for x in lens]
        tlen += lens[diffs.index(min(diffs))]  # first closest reference (reference tie-break)
    num, den = clipped_ngram_counts(p_ids, r_ids, n_gram)
    numerator += torch.from_numpy(num).to(numerator)
    denominator += torch.from_numpy(den).to(denominator)
    return preds_len + plen, target_len + tlen


def _bleu_score_compute(preds_len: Tensor, target_len: Tensor, numerator: Tensor, denominator: Tensor, n_gram: int,
                        weights: Sequence[float], smooth: bool) -> Tensor:
    device = numerator.device
    if min(numerator) == 0.0:
        return torch.tensor(0.0, device=device)
    if smooth:
        prec = (numerator + 1.0) / (denominator + 1.0)
        prec[0] = numerator[0] / denominator[0]
    else:
        prec = numerator / denominator
    geo = torch.exp(torch.sum(torch.tensor(weights, device=device) * torch.log(prec)))
    bp = torch.tensor(1.0, device=device) if preds_len > target_len else torch.exp(1 - (target_len / preds_len))
    return bp * geo


def _prepare(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]], n_gram: int,
             weights: Optional[Sequence[float]]) -> Tuple[Sequence[str], List[Sequence[str]], List[float]]:
    preds_ = [preds] if isinstance(preds, str) else preds
    target_ = [[t] if isinstance(t, str) else t for t in target]
    if len(preds_) != len(target_):
        raise ValueError(f"Corpus has different size {len(preds_)} != {len(target_)}")
    if weights is not None and len(weights) != n_gram:
        raise ValueError(f"List of weights has different weights than `n_gram`: {len(weights)} != {n_gram}")
    return preds_, target_, list(weights) if weights is not None else [1.0 / n_gram] * n_gram


def _bleu_with(tokenizer: Callable[[str], Sequence[str]], preds, target, n_gram, smooth, weights) -> Tensor:
    preds_, target_, weights = _prepare(preds, target, n_gram, weights)
    num, den = torch.zeros(n_gram), torch.zeros(n_gram)
    plen, tlen = _bleu_score_update(preds_, target_, num, den, torch.tensor(0.0), torch.tensor(0.0), n_gram,
                                    tokenizer)
    return _bleu_score_compute(plen, tlen, num, den, n_gram, weights, smooth)


def bleu_score(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]], n_gram: int = 4,
               smooth: bool = False, weights: Optional[Sequence[float]] = None) -> Tensor:
    """Corpus BLEU with whitespace tokenisation (``F/text/bleu.py``)."""
    return _bleu_with(_tokenize_fn, preds, target, n_gram, smooth, weights)


# ----------------------------------------------------------------------------------------------- sacrebleu tokenizers
# CJK ranges of the sacrebleu `zh` tokenizer
_CJK = (
    ("\u3400", "\u4db5"), ("\u4e00", "\u9fa5"), ("\u9fa6", "\u9fbb"), ("\uf900", "\ufa2d"), ("\ufa30", "\ufa6a"),
    ("\ufa70", "\ufad9"),
    # sacrebleu spells the two supplementary-plane ranges with 5 hex digits; Python's \u takes 4, so these are the
    # 2-character strings "\u2000" + "0" .. "\u2a6d" + "6" -- kept verbatim for identical tokenisation
    ("\u20000", "\u2a6d6"), ("\u2f800", "\u2fa1d"),
    ("\uff00", "\uffef"), ("\u2e80", "\u2eff"), ("\u3000", "\u303f"), ("\u31c0", "\u31ef"), ("\u2f00", "\u2fdf"),
    ("\u2ff0", "\u2fff"), ("\u3100", "\u312f"), ("\u31a0", "\u31bf"), ("\ufe10", "\ufe1f"), ("\ufe30", "\ufe4f"),
    ("\u2600", "\u26ff"), ("\u2700", "\u27bf"), ("\u3200", "\u32ff"), ("\u3300", "\u33ff"),
)

# mteval-v13a rules: split most ASCII punctuation, then periods / commas not between digits, then dash after digit
_MTEVAL_RULES = [
    (re.compile(r"([\{-\~\[-\` -\&\(-\+\:-\@\/])"), r" \1 "),
    (re.compile(r"([^0-9])([\.,])"), r"\1 \2 "),
    (re.compile(r"([\.,])([^0-9])"), r" \1 \2"),
    (re.compile(r"([0-9])(-)"), r"\1 \2 "),
]


@lru_cache(maxsize=1)
def _intl_rules():
    import regex

    return [
        (regex.compile(r"(\P{N})(\p{P})"), r"\1 \2 "),
        (regex.compile(r"(\p{P})(\P{N})"), r" \1 \2"),
        (regex.compile(r"(\p{S})"), r" \1 "),
    ]


def _apply(rules, line: str) -> str:
    for pat, rep in rules:
        line = pat.sub(rep, line)
    return " ".join(line.split())


def _tok_none(line: str) -> str:
    return line


def _tok_13a(line: str) -> str:
    line = line.replace("<skipped>", "").replace("-\n", "").replace("\n", " ")
    if "&" in line:
        for a, b in (("&quot;", '"'), ("&amp;", "&"), ("&lt;", "<"), ("&gt;", ">")):
            line = line.replace(a, b)
    return _apply(_MTEVAL_RULES, f" {line} ")


def _is_cjk(ch: str) -> bool:
    return any(lo <= ch <= hi for lo, hi in _CJK)


def _tok_zh(line: str) -> str:
    return _apply(_MTEVAL_RULES, "".join(f" {c} " if _is_cjk(c) else c for c in line.strip()))


def _tok_intl(line: str) -> str:
    return _apply(_intl_rules(), line)


def _tok_char(line: str) -> str:
    return " ".join(line)


def _tok_ja_mecab(line: str) -> str:
    import ipadic
    import MeCab

    return MeCab.Tagger(ipadic.MECAB_ARGS + " -Owakati").parse(line.strip()).strip()


def _tok_ko_mecab(line: str) -> str:
    import mecab_ko
    import mecab_ko_dic

    return mecab_ko.Tagger(mecab_ko_dic.MECAB_ARGS + " -Owakati").parse(line.strip()).strip()


@lru_cache(maxsize=2)
def _spm(kind: str):
    import sentencepiece

    path = os.path.join(_FLORES_LOCAL_DIR, _FLORES_FILES[kind])
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"`{kind}` tokenization needs the FLORES sentencepiece model at {path}; this build never downloads files,"
            " place the model there manually."
        )
    proc = sentencepiece.SentencePieceProcessor()
    proc.Load(path)
    return proc


def _tok_flores(kind: str) -> Callable[[str], str]:
    return lambda line: " ".join(_spm(kind).EncodeAsPieces(line))


_TOKENIZERS: Dict[str, Callable[[str], str]] = {
    "none": _tok_none, "13a": _tok_13a, "zh": _tok_zh, "intl": _tok_intl, "char": _tok_char,
    "ja-mecab": _tok_ja_mecab, "ko-mecab": _tok_ko_mecab, "flores101": _tok_flores("flores101"),
    "flores200": _tok_flores("flores200"),
}
_REQUIRES = {"intl": ("regex",), "ja-mecab": ("MeCab", "ipadic"), "ko-mecab": ("mecab_ko", "mecab_ko_dic"),
             "flores101": ("sentencepiece",), "flores200": ("sentencepiece",)}


class _SacreBLEUTokenizer:
    """SacreBLEU tokenizer selector (``F/text/sacre_bleu.py:74``)."""

    def __init__(self, tokenize: _TokenizersLiteral, lowercase: bool = False) -> None:
        self._check_tokenizers_validity(tokenize)
        self.tokenize_fn = _TOKENIZERS[tokenize]
        self.lowercase = lowercase

    def __call__(self, line: str) -> Sequence[str]:
        out = self.tokenize_fn(line)
        return (out.lower() if self.lowercase else out).split()

    @classmethod
    def tokenize(cls, line: str, tokenize: _TokenizersLiteral, lowercase: bool = False) -> Sequence[str]:
        return cls(tokenize, lowercase)(line)

    @staticmethod
    def _check_tokenizers_validity(tokenize: str) -> None:
        if tokenize not in _TOKENIZERS:
            raise ValueError(f"Unsupported tokenizer selected. Please, choose one of {list(_TOKENIZERS)}")
        missing = [m for m in _REQUIRES.get(tokenize, ()) if importlib.util.find_spec(m) is None]
        if missing:
            raise ModuleNotFoundError(f"`'{tokenize}'` tokenization requires that {missing} are installed.")


def sacre_bleu_score(preds: Sequence[str], target: Sequence[Sequence[str]], n_gram: int = 4, smooth: bool = False,
                     tokenize: _TokenizersLiteral = "13a", lowercase: bool = False,
                     weights: Optional[Sequence[float]] = None) -> Tensor:
    """BLEU with SacreBLEU tokenisation (``F/text/sacre_bleu.py``)."""
    return _bleu_with(_SacreBLEUTokenizer(tokenize, lowercase), preds, target, n_gram, smooth, weights)
