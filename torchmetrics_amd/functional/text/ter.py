"""Translation edit rate (reference ``F/text/ter.py``, tercom semantics as in sacrebleu).

Greedy shift search over the beam edit distance of :class:`~torchmetrics_amd.functional.text.helper.BeamEditDistance`
(prefix-trie row cache, operation trace -> alignment).  Candidate ordering, corner cases and the candidate budget
follow tercom so scores are identical.
"""
import re
from functools import lru_cache
from typing import Iterator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd.functional.text.helper import BeamEditDistance, _validate_inputs, flip_trace, trace_to_alignment

_MAX_SHIFT_SIZE = 10
_MAX_SHIFT_DIST = 50
_MAX_SHIFT_CANDIDATES = 1000

_ASIAN_PUNCT = r"([\u3001\u3002\u3008-\u3011\u3014-\u301f\uff61-\uff65\u30fb])"
_FULL_WIDTH_PUNCT = r"([\uff0e\uff0c\uff1f\uff1a\uff1b\uff01\uff02\uff08\uff09])"
_WESTERN_RULES = [(re.compile(p), r) for p, r in (
    (r"\n-", ""), (r"\n", " "), (r"&quot;", '"'), (r"&amp;", "&"), (r"&lt;", "<"), (r"&gt;", ">"),
    (r"([{-~[-` -&(-+:-@/])", r" \1 "), (r"'s ", r" 's "), (r"'s$", r" 's"), (r"([^0-9])([\.,])", r"\1 \2 "),
    (r"([\.,])([^0-9])", r" \1 \2"), (r"([0-9])(-)", r"\1 \2 "),
)]
_ASIAN_RULES = [(re.compile(p), r) for p, r in (
    (r"([\u4e00-\u9fff\u3400-\u4dbf])", r" \1 "),  # CJK ideographs
    (r"([\u31c0-\u31ef\u2e80-\u2eff])", r" \1 "),  # strokes, radicals
    (r"([\u3300-\u33ff\uf900-\ufaff\ufe30-\ufe4f])", r" \1 "),
    (r"([\u3200-\u3f22])", r" \1 "),
    (r"(^|^[\u3040-\u309f])([\u3040-\u309f]+)(?=$|^[\u3040-\u309f])", r"\1 \2 "),  # hiragana
    (r"(^|^[\u30a0-\u30ff])([\u30a0-\u30ff]+)(?=$|^[\u30a0-\u30ff])", r"\1 \2 "),  # katakana
    (r"(^|^[\u31f0-\u31ff])([\u31f0-\u31ff]+)(?=$|^[\u31f0-\u31ff])", r"\1 \2 "),
    (_ASIAN_PUNCT, r" \1 "),
    (_FULL_WIDTH_PUNCT, r" \1 "),
)]
_PUNCT = re.compile(r"[\.,\?:;!\"\(\)]")


class _TercomTokenizer:
    """Tercom normaliser (``F/text/ter.py:45``)."""

    def __init__(self, normalize: bool = False, no_punctuation: bool = False, lowercase: bool = True,
                 asian_support: bool = False) -> None:
        self.normalize = normalize
        self.no_punctuation = no_punctuation
        self.lowercase = lowercase
        self.asian_support = asian_support
        self._call = lru_cache(maxsize=2**16)(self._tokenize)

    def __call__(self, sentence: str) -> str:
        return self._call(sentence)

    def _tokenize(self, sentence: str) -> str:
        if not sentence:
            return ""
        if self.lowercase:
            sentence = sentence.lower()
        if self.normalize:
            sentence = f" {sentence} "
            for pat, rep in _WESTERN_RULES:
                sentence = pat.sub(rep, sentence)
            if self.asian_support:
                for pat, rep in _ASIAN_RULES:
                    sentence = pat.sub(rep, sentence)
        if self.no_punctuation:
            sentence = _PUNCT.sub("", sentence)
            if self.asian_support:
                sentence = re.sub(_FULL_WIDTH_PUNCT, "", re.sub(_ASIAN_PUNCT, "", sentence))
        return " ".join(sentence.split())


def _shift_candidates(hyp: List[str], ref: List[str]) -> Iterator[Tuple[int, int, int]]:
    """(hyp_start, ref_start, length) of equal spans, |start distance| <= 50, length < 10."""
    for hs in range(len(hyp)):
        for rs in range(len(ref)):
            if abs(rs - hs) > _MAX_SHIFT_DIST:
                continue
            for length in range(1, _MAX_SHIFT_SIZE):
                if hyp[hs + length - 1] != ref[rs + length - 1]:
                    break
                yield hs, rs, length
                if len(hyp) == hs + length or len(ref) == rs + length:
                    break


def _move(words: List[str], start: int, length: int, target: int) -> List[str]:
    """Move ``words[start:start+length]`` so it begins before position ``target`` of the original list."""
    span = words[start:start + length]
    if target < start:
        return words[:target] + span + words[target:start] + words[start + length:]
    if target > start + length:
        return words[:start] + words[start + length:target] + span + words[target:]
    return words[:start] + words[start + length:length + target] + span + words[length + target:]


def _best_shift(hyp: List[str], ref: List[str], ed: BeamEditDistance, checked: int) -> Tuple[int, List[str], int]:
    dist, trace = ed(hyp)
    align, ref_err, hyp_err = trace_to_alignment(flip_trace(trace))
    best: Optional[tuple] = None
    for hs, rs, length in _shift_candidates(hyp, ref):
        if (sum(hyp_err[hs:hs + length]) == 0 or sum(ref_err[rs:rs + length]) == 0
                or hs <= align[rs] < hs + length):
            continue
        prev = -1
        for off in range(-1, length):
            if rs + off == -1:
                idx = 0
            elif rs + off in align:
                idx = align[rs + off] + 1
            else:
                break
            if idx == prev:
                continue
            prev = idx
            shifted = _move(hyp, hs, length, idx)
            # larger gain, then longer span, then earlier hyp start, then earlier target position
            cand = (dist - ed(shifted)[0], length, -hs, -idx, shifted)
            checked += 1
            if best is None or cand > best:
                best = cand
        if checked >= _MAX_SHIFT_CANDIDATES:
            break
    if best is None:
        return 0, hyp, checked
    return best[0], best[4], checked


def _translation_edit_rate(hyp: List[str], ref: List[str]) -> Tensor:
    """Shifts + edits turning ``hyp`` into ``ref`` (tercom greedy search)."""
    if len(ref) == 0:
        return torch.tensor(0.0)
    ed = BeamEditDistance(ref)
    shifts = checked = 0
    words = hyp
    while True:
        gain, shifted, checked = _best_shift(words, ref, ed, checked)
        if checked >= _MAX_SHIFT_CANDIDATES or gain <= 0:
            break
        shifts += 1
        words = shifted
    return torch.tensor(float(shifts + ed(words)[0]))


def _compute_sentence_statistics(pred_words: List[str], target_words: List[List[str]]) -> Tuple[Tensor, Tensor]:
    """(fewest edits over references, average reference length).  As in the reference (and sacrebleu), the shift
    search runs on the *reference* words against the hypothesis (``F/text/ter.py:446``)."""
    best = torch.tensor(2e16)
    tot = 0.0
    for tgt in target_words:
        edits = _translation_edit_rate(tgt, pred_words)
        tot += len(tgt)
        if edits < best:
            best = edits
    return best, torch.tensor(tot / len(target_words))


def _compute_ter_score_from_statistics(num_edits: Tensor, tgt_length: Tensor) -> Tensor:
    if tgt_length > 0 and num_edits > 0:
        return num_edits / tgt_length
    if tgt_length == 0 and num_edits > 0:
        return torch.tensor(1.0)
    return torch.tensor(0.0)


def _ter_update(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]],
                tokenizer: _TercomTokenizer, total_num_edits: Tensor, total_tgt_length: Tensor,
                sentence_ter: Optional[List[Tensor]] = None) -> Tuple[Tensor, Tensor, Optional[List[Tensor]]]:
    target, preds = _validate_inputs(target, preds)
    for pred, tgt in zip(preds, target):
        tgt_words = [tokenizer(t.rstrip()).split() for t in tgt]
        pred_words = tokenizer(pred.rstrip()).split()
        num_edits, tgt_length = _compute_sentence_statistics(pred_words, tgt_words)
        total_num_edits = total_num_edits + num_edits.to(total_num_edits)
        total_tgt_length = total_tgt_length + tgt_length.to(total_tgt_length)
        if sentence_ter is not None:
            sentence_ter.append(_compute_ter_score_from_statistics(num_edits, tgt_length).unsqueeze(0))
    return total_num_edits, total_tgt_length, sentence_ter


def _ter_compute(total_num_edits: Tensor, total_tgt_length: Tensor) -> Tensor:
    return _compute_ter_score_from_statistics(total_num_edits, total_tgt_length)


def _check_ter_flags(**flags: bool) -> None:
    for name, val in flags.items():
        if not isinstance(val, bool):
            raise ValueError(f"Expected argument `{name}` to be of type boolean but got {val}.")


def translation_edit_rate(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]],
                          normalize: bool = False, no_punctuation: bool = False, lowercase: bool = True,
                          asian_support: bool = False, return_sentence_level_score: bool = False
                          ) -> Union[Tensor, Tuple[Tensor, List[Tensor]]]:
    """Corpus TER: (shifts + edits) / average reference length (``F/text/ter.py:519``)."""
    _check_ter_flags(normalize=normalize, no_punctuation=no_punctuation, lowercase=lowercase,
                     asian_support=asian_support)
    tok = _TercomTokenizer(normalize, no_punctuation, lowercase, asian_support)
    sentence_ter: Optional[List[Tensor]] = [] if return_sentence_level_score else None
    edits, length, sentence_ter = _ter_update(preds, target, tok, torch.tensor(0.0), torch.tensor(0.0), sentence_ter)
    score = _ter_compute(edits, length)
    if sentence_ter:
        return score, sentence_ter
    return score
