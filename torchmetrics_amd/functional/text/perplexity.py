"""Perplexity (reference ``F/text/perplexity.py``) on the fused single-pass token-NLL kernel
(:func:`torchmetrics_amd.ops.token_nll`): no ``[B*S, V]`` probability tensor is materialised."""
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops


def _check_shape_and_type_consistency(preds: Tensor, target: Tensor) -> None:
    if len(preds.shape) != 3:
        raise ValueError(
            "Input tensor `preds` is expected to have 3 dimensions, [batch_size, seq_len, vocab_size],"
            f" but got {len(preds.shape)}."
        )
    if len(target.shape) != 2:
        raise ValueError(
            "Input tensor `target` is expected to have 2 dimensions, [batch_size, seq_len],"
            f" but got {len(target.shape)}."
        )
    if preds.shape[:2] != target.shape:
        raise ValueError(
            "Input tensors `preds` and `target` are expected to have equaling first two dimensions,"
            f" [batch_size, seq_len], but got {preds.shape[:2]} and {target.shape}."
        )
    if not preds.is_floating_point():
        raise TypeError(f"Input tensor `preds` is expected to be of floating point type but got {preds.dtype}.")
    if target.dtype != torch.int64:
        raise TypeError(f"Input tensor `target` is expected to be of a type {torch.int64} but got {target.dtype}.")


def _perplexity_update(preds: Tensor, target: Tensor, ignore_index: Optional[int] = None,
                       flag: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """(sum of token NLL, number of scored tokens)."""
    _check_shape_and_type_consistency(preds, target)
    logits = preds.reshape(-1, preds.shape[-1])
    tgt = target.reshape(-1)
    nll = ops.token_nll(logits, tgt, ignore_index, flag)
    count = tgt.numel() if ignore_index is None else (tgt != ignore_index).sum()
    total = nll.sum()
    if preds.dtype == torch.float64:
        total = total.double()
    return total, torch.as_tensor(count, device=preds.device)


def _perplexity_compute(total: Tensor, count: Tensor) -> Tensor:
    return torch.exp(total / count)


def perplexity(preds: Tensor, target: Tensor, ignore_index: Optional[int] = None) -> Tensor:
    """exp(mean token negative log-likelihood) of ``preds [B, S, V]`` logits (``F/text/perplexity.py``)."""
    total, count = _perplexity_update(preds, target, ignore_index)
    return _perplexity_compute(total, count)
