"""Shared plumbing for the model-based text metrics (BERTScore, InfoLM): tokenisation, IDF tables and a
length-sorted batched model runner (reference ``F/text/helper_embedding_metric.py``).

Sentences are processed in length-sorted batches trimmed to the batch's longest sequence (less padding work for the
encoder), and results are scattered back to the *original* order with the inverse permutation.  (The reference
re-indexes its outputs with the forward sort permutation and sorts predictions and references independently,
``F/text/bert.py:418-425``, which pairs sentences correctly only when both sides sort identically; here pairs are
always (preds[i], target[i]).)
"""
import math
from collections import Counter
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import torch
from torch import Tensor


def tokenize(text: List[str], tokenizer: Any, max_length: int, own_tokenizer: bool = False,
             truncation: bool = True) -> Dict[str, Tensor]:
    """HF call convention ``tokenizer(text, padding=..., max_length=..., ...)``; a user's own tokenizer is called as
    ``tokenizer(text, max_length)`` and must return ``input_ids`` / ``attention_mask``."""
    if not own_tokenizer:
        out = tokenizer(text, padding="max_length", max_length=max_length, truncation=truncation, return_tensors="pt")
    else:
        try:
            out = tokenizer(text, max_length)
        except BaseException as ex:  # noqa: BLE001  (surface any user tokenizer failure uniformly)
            raise RuntimeError(f"Tokenization was not successful: {ex}") from ex
    return {"input_ids": out["input_ids"], "attention_mask": out["attention_mask"]}


def idf_table(input_ids: Tensor) -> Tuple[Dict[int, float], float]:
    """Inverse document frequencies ``log((N + 1) / (df + 1))`` over the rows of ``input_ids`` and the default
    value ``log(N + 1)`` for unseen tokens."""
    n = input_ids.shape[0]
    df: Counter = Counter()
    for row in input_ids.tolist():
        df.update(set(row))
    return {tok: math.log((n + 1) / (c + 1)) for tok, c in df.items()}, math.log(n + 1)


def idf_weights(input_ids: Tensor, table: Dict[int, float], default: float) -> Tensor:
    flat = input_ids.reshape(-1).tolist()
    return torch.tensor([table.get(t, default) for t in flat], dtype=torch.float32).reshape(input_ids.shape)


def sorted_batches(attention_mask: Tensor, batch_size: int) -> Iterator[Tuple[Tensor, int]]:
    """Yield (row indices of a batch in ascending-length order, trimmed length)."""
    lengths = attention_mask.sum(1)
    order = torch.argsort(lengths, stable=True)
    for s in range(0, order.numel(), batch_size):
        idx = order[s:s + batch_size]
        yield idx, max(int(lengths[idx].max().item()), 1)


def run_sorted(attention_mask: Tensor, batch_size: int, fn: Callable[[Tensor, int], Tensor],
               verbose: bool = False) -> Tensor:
    """Apply ``fn(rows, trimmed_len) -> [rows, ...]`` to length-sorted batches; results are returned in original row
    order (rows padded along dim 1 to the longest batch when ``fn`` returns per-token tensors)."""
    batches = list(sorted_batches(attention_mask, batch_size))
    if verbose:
        import tqdm

        batches = tqdm.auto.tqdm(batches)
    outs, rows = [], []
    for idx, ln in batches:
        outs.append(fn(idx, ln))
        rows.append(idx)
    if not outs:
        return torch.zeros(0)
    if outs[0].dim() >= 2 and any(o.shape[1] != outs[0].shape[1] for o in outs):
        width = max(o.shape[1] for o in outs)
        outs = [torch.nn.functional.pad(o, [0, 0] * (o.dim() - 2) + [0, width - o.shape[1]]) for o in outs]
    cat = torch.cat(outs)
    res = torch.empty_like(cat)
    res[torch.cat(rows).to(cat.device)] = cat
    return res


def progress(iterable: Any, verbose: bool) -> Any:
    if verbose:
        import tqdm

        return tqdm.auto.tqdm(iterable)
    return iterable
