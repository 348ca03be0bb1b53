"""Extended edit distance (reference ``F/text/eed.py``; RWTH EED).

The character DP with CDER jumps runs in the native host op ``tm_amd::eed_score`` when the library is loaded (exact
sequential double-precision semantics of the reference, multithreaded over sentence pairs), with a pure-Python
fallback of the same recurrence.
"""
import re
import unicodedata
from math import inf
from typing import List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.text.helper import _validate_inputs


def _eed_function(hyp: str, ref: str, alpha: float = 2.0, rho: float = 0.3, deletion: float = 0.2,
                  insertion: float = 1.0) -> float:
    """EED of one (hypothesis, reference) character pair (CDER-initialised DP, jump on reference blanks)."""
    n = len(hyp)
    visits = [-1] * (n + 1)
    row = [1.0] * (n + 1)
    row[0] = 0.0
    for w in range(len(ref)):
        rc = ref[w]
        nxt = [0.0] * (n + 1)
        nxt[0] = row[0] + 1.0
        for i in range(1, n + 1):
            nxt[i] = min(nxt[i - 1] + deletion, row[i - 1] + (hyp[i - 1] != rc), row[i] + insertion)
        best = min(nxt)
        k = nxt.index(best)
        visits[k] += 1
        if rc == " ":
            jump = alpha + best
            nxt = [x if x < jump else jump for x in nxt]
        row = nxt
    coverage = rho * sum(x if x >= 0 else 1 for x in visits)
    return min(1, (row[-1] + coverage) / (float(len(ref)) + coverage))


_EN_PUNCT = ((".", " ."), ("!", " !"), ("?", " ?"), (",", " ,"))
_EN_RE = [(re.compile(r"\s+"), r" "), (re.compile(r"(\d) ([.,]) (\d)"), r"\1\2\3"),
          (re.compile(r"(Dr|Jr|Prof|Rev|Gen|Mr|Mt|Mrs|Ms) ."), r"\1.")]
_EN_ABBR = (("e . g .", "e.g."), ("i . e .", "i.e."), ("U . S .", "U.S."))


def _preprocess_en(sentence: str) -> str:
    if not isinstance(sentence, str):
        raise ValueError(f"Only strings allowed during preprocessing step, found {type(sentence)} instead")
    sentence = sentence.rstrip()
    for a, b in _EN_PUNCT:
        sentence = sentence.replace(a, b)
    for pat, rep in _EN_RE:
        sentence = pat.sub(rep, sentence)
    for a, b in _EN_ABBR:
        sentence = sentence.replace(a, b)
    return " " + sentence + " "


def _preprocess_ja(sentence: str) -> str:
    if not isinstance(sentence, str):
        raise ValueError(f"Only strings allowed during preprocessing step, found {type(sentence)} instead")
    return unicodedata.normalize("NFKC", sentence.rstrip())


def _preprocess_sentences(preds, target, language):
    target, preds = _validate_inputs(hypothesis_corpus=preds, ref_corpus=target)
    if language == "en":
        fn = _preprocess_en
    elif language == "ja":
        fn = _preprocess_ja
    else:
        raise ValueError(f"Expected argument `language` to either be `en` or `ja` but got {language}")
    return [fn(p) for p in preds], [[fn(r) for r in refs] for refs in target]


def _eed_scores(pairs: List[Tuple[str, str]], alpha: float, rho: float, deletion: float,
                insertion: float) -> List[float]:
    if pairs and ops.native_available():
        return ops.eed_scores([p for p, _ in pairs], [r for _, r in pairs], alpha, rho, deletion, insertion)
    return [_eed_function(h, r, alpha, rho, deletion, insertion) for h, r in pairs]


def _eed_update(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]],
                language: Literal["en", "ja"] = "en", alpha: float = 2.0, rho: float = 0.3, deletion: float = 0.2,
                insertion: float = 1.0, sentence_eed: Optional[List[Tensor]] = None) -> List[Tensor]:
    preds, target = _preprocess_sentences(preds, target, language)
    if sentence_eed is None:
        sentence_eed = []
    if 0 in (len(preds), len(target[0])):
        return sentence_eed
    pairs, owner = [], []
    for s, (hyp, refs) in enumerate(zip(preds, target)):
        for ref in refs:
            pairs.append((hyp, ref))
            owner.append(s)
    scores = _eed_scores(pairs, alpha, rho, deletion, insertion)
    best = [inf] * min(len(preds), len(target))
    for s, v in zip(owner, scores):
        if v < best[s]:
            best[s] = v
    sentence_eed.extend(torch.tensor(b) for b in best)
    return sentence_eed


def _eed_compute(sentence_level_scores: List[Tensor]) -> Tensor:
    if len(sentence_level_scores) == 0:
        return torch.tensor(0.0)
    return sum(sentence_level_scores) / torch.tensor(len(sentence_level_scores))


def _check_eed_params(alpha: float, rho: float, deletion: float, insertion: float) -> None:
    for name, val in zip(["alpha", "rho", "deletion", "insertion"], [alpha, rho, deletion, insertion]):
        if not isinstance(val, float) or val < 0:
            raise ValueError(f"Parameter `{name}` is expected to be a non-negative float.")


def extended_edit_distance(preds: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]],
                           language: Literal["en", "ja"] = "en", return_sentence_level_score: bool = False,
                           alpha: float = 2.0, rho: float = 0.3, deletion: float = 0.2, insertion: float = 1.0
                           ) -> Union[Tensor, Tuple[Tensor, Tensor]]:
    """Average sentence EED (best over references), ``F/text/eed.py:352``."""
    _check_eed_params(alpha, rho, deletion, insertion)
    scores = _eed_update(preds, target, language, alpha, rho, deletion, insertion)
    avg = _eed_compute(scores)
    if return_sentence_level_score:
        return avg, torch.stack(scores)
    return avg
