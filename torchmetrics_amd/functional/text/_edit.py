"""Token-id packing + batched edit distance shared by the ASR error rates and EditDistance.

Strings are tokenised on the host (words: whitespace split mapped through a per-call vocabulary; characters: their
code points), packed into one int32 id buffer with int64 offsets, and all pairs of a batch are solved by a single
call of :func:`torchmetrics_amd.ops.levenshtein` (wave-per-pair HIP kernel on ROCm tensors, native multithreaded DP
on the host) instead of the reference's per-pair Python DP (``F/text/helper.py:329``).
"""
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd import ops


def _as_list(x: Union[str, Sequence[str]]) -> List[str]:
    return [x] if isinstance(x, str) else list(x)


def _char_ids(text: str) -> np.ndarray:
    return np.frombuffer(text.encode("utf-32-le"), dtype=np.uint32).astype(np.int32)


def _word_ids(tokens: Sequence[str], vocab: Dict[str, int]) -> np.ndarray:
    return np.fromiter((vocab.setdefault(t, len(vocab)) for t in tokens), dtype=np.int32, count=len(tokens))


def _pack(seqs: List[np.ndarray]) -> Tuple[Tensor, Tensor, int]:
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
    off = np.zeros(len(seqs) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    ids = np.concatenate(seqs) if seqs and off[-1] else np.zeros(0, dtype=np.int32)
    return torch.from_numpy(ids.astype(np.int32, copy=False)), torch.from_numpy(off), int(lens.max()) if len(lens) else 0


def tokenize_pairs(preds: List[str], target: List[str], level: str) -> Tuple[List[np.ndarray], List[np.ndarray]]:
    if level == "char":
        return [_char_ids(p) for p in preds], [_char_ids(t) for t in target]
    vocab: Dict[str, int] = {}
    return [_word_ids(p.split(), vocab) for p in preds], [_word_ids(t.split(), vocab) for t in target]


def batched_edit_distance(pred_ids: List[np.ndarray], ref_ids: List[np.ndarray], substitution_cost: int = 1,
                          beam: bool = False, device: Optional[torch.device] = None) -> Tensor:
    """``[B]`` int64 edit distances transforming each prediction into its reference."""
    p, po, _ = _pack(pred_ids)
    r, ro, rmax = _pack(ref_ids)
    if device is not None and torch.device(device).type == "cuda":
        dev = torch.device(device)
        p, po, r, ro = (t.pin_memory().to(dev, non_blocking=True) for t in (p, po, r, ro))
    return ops.levenshtein(p, po, r, ro, 1, 1, int(substitution_cost), beam, rmax)
