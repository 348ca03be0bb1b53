"""Shared text-metric helpers: corpus validation and the tercom beam edit distance with operation trace
(reference ``F/text/helper.py``)."""
import math
from typing import Dict, List, Sequence, Tuple, Union

_BEAM_WIDTH = 25
_MAX_CACHE_SIZE = 10000
_INF = 1 << 60

# operation codes of a trace (rewriting the hypothesis into the reference)
OP_NOTHING, OP_SUBSTITUTE, OP_INSERT, OP_DELETE = "n", "s", "i", "d"


def _validate_inputs(ref_corpus: Union[Sequence[str], Sequence[Sequence[str]]],
                     hypothesis_corpus: Union[str, Sequence[str]]) -> Tuple[Sequence[Sequence[str]], Sequence[str]]:
    """Normalise ``(references, hypotheses)`` to ``(list of reference lists, list of hypotheses)``."""
    if isinstance(hypothesis_corpus, str):
        hypothesis_corpus = [hypothesis_corpus]
    if all(isinstance(ref, str) for ref in ref_corpus):
        ref_corpus = [ref_corpus] if len(hypothesis_corpus) == 1 else [[ref] for ref in ref_corpus]  # type: ignore
    if hypothesis_corpus and all(ref for ref in ref_corpus) and len(ref_corpus) != len(hypothesis_corpus):
        raise ValueError(f"Corpus has different size {len(ref_corpus)} != {len(hypothesis_corpus)}")
    return ref_corpus, hypothesis_corpus


class BeamEditDistance:
    """Tercom beam-limited Levenshtein distance to a fixed reference with an operation trace.

    Rows of the DP are cached in a prefix trie keyed by hypothesis tokens, so TER's many shifted candidates (which
    share long prefixes) only recompute their suffix rows.  Costs: insert / delete 1, substitute ``op_substitute``.
    Tie preference (tercom): keep / substitute, then delete, then insert.
    """

    def __init__(self, reference: Sequence, op_insert: int = 1, op_delete: int = 1, op_substitute: int = 1) -> None:
        self.ref = list(reference)
        self.rlen = len(self.ref)
        self.ins, self.dele, self.sub = op_insert, op_delete, op_substitute
        self._trie: Dict = {}
        self._cached = 0
        self._row0 = ([j * self.ins for j in range(self.rlen + 1)], [OP_INSERT] * (self.rlen + 1))

    def __call__(self, hyp: Sequence) -> Tuple[int, str]:
        hyp = list(hyp)
        plen = len(hyp)
        rows = [self._row0]
        node = self._trie
        for tok in hyp:  # longest cached prefix
            nxt = node.get(tok)
            if nxt is None:
                break
            node, row = nxt
            rows.append(row)
        start = len(rows) - 1
        ratio = self.rlen / plen if plen else 1.0
        width = math.ceil(ratio / 2 + _BEAM_WIDTH) if ratio / 2 > _BEAM_WIDTH else _BEAM_WIDTH
        ref, ins, dele, sub = self.ref, self.ins, self.dele, self.sub
        for i in range(start + 1, plen + 1):
            prev_c = rows[i - 1][0]
            cost = [_INF] * (self.rlen + 1)
            op = ["?"] * (self.rlen + 1)
            diag = math.floor(i * ratio)
            lo = max(0, diag - width)
            hi = self.rlen + 1 if i == plen else min(self.rlen + 1, diag + width)
            tok = hyp[i - 1]
            for j in range(lo, hi):
                if j == 0:
                    cost[0], op[0] = prev_c[0] + dele, OP_DELETE
                    continue
                if tok == ref[j - 1]:
                    best, bop = prev_c[j - 1], OP_NOTHING
                else:
                    best, bop = prev_c[j - 1] + sub, OP_SUBSTITUTE
                c = prev_c[j] + dele
                if c < best:
                    best, bop = c, OP_DELETE
                c = cost[j - 1] + ins
                if c < best:
                    best, bop = c, OP_INSERT
                cost[j], op[j] = best, bop
            rows.append((cost, op))
        self._add_cache(hyp, rows, start)
        # backtrace
        trace = []
        i, j = plen, self.rlen
        while i > 0 or j > 0:
            o = rows[i][1][j]
            trace.append(o)
            if o in (OP_NOTHING, OP_SUBSTITUTE):
                i, j = i - 1, j - 1
            elif o == OP_INSERT:
                j -= 1
            elif o == OP_DELETE:
                i -= 1
            else:
                raise ValueError(f"Unknown operation {o!r}")
        return rows[plen][0][self.rlen], "".join(reversed(trace))

    def _add_cache(self, hyp: List, rows: List, start: int) -> None:
        if self._cached >= _MAX_CACHE_SIZE:
            return
        node = self._trie
        for tok in hyp[:start]:
            node = node[tok][0]
        for k in range(start, len(hyp)):
            tok = hyp[k]
            if tok not in node:
                node[tok] = ({}, rows[k + 1])
                self._cached += 1
            node = node[tok][0]


def flip_trace(trace: str) -> str:
    """Rewrite recipe b->a from a->b: swap insertions and deletions."""
    return trace.translate(str.maketrans({OP_INSERT: OP_DELETE, OP_DELETE: OP_INSERT}))


def trace_to_alignment(trace: str) -> Tuple[Dict[int, int], List[int], List[int]]:
    """(reference position -> hypothesis position, reference error flags, hypothesis error flags)."""
    rpos = hpos = -1
    ref_err: List[int] = []
    hyp_err: List[int] = []
    align: Dict[int, int] = {}
    for o in trace:
        if o == OP_NOTHING or o == OP_SUBSTITUTE:
            hpos += 1
            rpos += 1
            align[rpos] = hpos
            e = 0 if o == OP_NOTHING else 1
            ref_err.append(e)
            hyp_err.append(e)
        elif o == OP_INSERT:
            hpos += 1
            hyp_err.append(1)
        elif o == OP_DELETE:
            rpos += 1
            align[rpos] = hpos
            ref_err.append(1)
        else:
            raise ValueError(f"Unknown operation {o!r}.")
    return align, ref_err, hyp_err
