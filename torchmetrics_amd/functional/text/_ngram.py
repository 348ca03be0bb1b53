"""Vectorised clipped n-gram statistics (BLEU family) on integer token ids.

The reference builds a ``collections.Counter`` of n-gram tuples per sentence and intersects / unions them in Python
(``F/text/bleu.py:27-90``).  Here every n-gram of every sentence becomes one row ``(sentence, ref, w_1 .. w_n)`` of an
int64 matrix; counting is ``np.unique(axis=0)``, the max over references is a ``np.maximum.at`` on the
``(sentence, n-gram)`` inverse index, and clipping is a sorted-key intersection -- O(total tokens log) with no Python
loop over n-grams.
"""
from typing import Dict, List, Sequence, Tuple

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view


def ids_of(tokens: Sequence[str], vocab: Dict[str, int]) -> np.ndarray:
    return np.fromiter((vocab.setdefault(t, len(vocab)) for t in tokens), dtype=np.int64, count=len(tokens))


def _windows(seqs: List[np.ndarray], tags: np.ndarray, n: int) -> np.ndarray:
    """Rows ``[tag..., w_1..w_n]`` for every length-n window of every sequence (tags: [S, k])."""
    blocks = []
    for s, seq in enumerate(seqs):
        if len(seq) >= n:
            w = sliding_window_view(seq, n)
            blocks.append(np.concatenate([np.broadcast_to(tags[s], (w.shape[0], tags.shape[1])), w], axis=1))
    if not blocks:
        return np.zeros((0, tags.shape[1] + n), dtype=np.int64)
    return np.concatenate(blocks, axis=0)


def _row_keys(rows: np.ndarray) -> np.ndarray:
    """Exact 1-D sortable keys for int64 rows (contiguous void view)."""
    rows = np.ascontiguousarray(rows)
    return rows.view(np.dtype((np.void, rows.dtype.itemsize * rows.shape[1]))).ravel()


def clipped_ngram_counts(preds: List[np.ndarray], refs: List[List[np.ndarray]],
                         n_gram: int) -> Tuple[np.ndarray, np.ndarray]:
    """(numerator[n], denominator[n]): clipped matches and total prediction n-grams for n = 1..n_gram."""
    num = np.zeros(n_gram, dtype=np.float64)
    den = np.zeros(n_gram, dtype=np.float64)
    flat_refs = [r for rs in refs for r in rs]
    ref_tags = np.array([(s, k) for s, rs in enumerate(refs) for k in range(len(rs))], dtype=np.int64).reshape(-1, 2)
    pred_tags = np.arange(len(preds), dtype=np.int64)[:, None]
    for n in range(1, n_gram + 1):
        prow = _windows(preds, pred_tags, n)
        den[n - 1] = prow.shape[0]
        if prow.shape[0] == 0:
            continue
        pk, pc = np.unique(prow, axis=0, return_counts=True)
        rrow = _windows(flat_refs, ref_tags, n)
        if rrow.shape[0] == 0:
            continue
        rk, rc = np.unique(rrow, axis=0, return_counts=True)  # per (sentence, ref, ngram)
        # max over references: drop the ref column and fold equal (sentence, ngram) keys
        sk, inv = np.unique(np.delete(rk, 1, axis=1), axis=0, return_inverse=True)
        rmax = np.zeros(sk.shape[0], dtype=np.int64)
        np.maximum.at(rmax, inv.ravel(), rc)
        _, ip, ir = np.intersect1d(_row_keys(pk), _row_keys(sk), assume_unique=True, return_indices=True)
        num[n - 1] = np.minimum(pc[ip], rmax[ir]).sum()
    return num, den
