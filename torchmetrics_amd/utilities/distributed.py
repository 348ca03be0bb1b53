"""Legacy reductions + the reference-compatible per-tensor gather.

* ``reduce`` / ``class_reduce``: parity with reference ``S/utilities/distributed.py:22,45``.
* ``gather_all_tensors``: the *user-visible* per-tensor gather contract (reference ``:97-147``). It is kept for
  users who pass it (or their own function) as ``dist_sync_fn``. The framework's default sync does NOT use it: a
  ``Metric`` with ``dist_sync_fn=None`` goes through the bucketed RCCL engine in
  :mod:`torchmetrics_amd.parallel.sync`, which all-reduces SUM/MEAN/MAX/MIN states in one collective per
  (op, dtype) bucket and all-gathers CAT states in one collective per dtype, with no barriers.
"""
from typing import Any, List, Optional

import torch
from torch import Tensor
from torch.nn import functional as F


def reduce(x: Tensor, reduction: Optional[str]) -> Tensor:
    """Reduce ``x`` by ``'elementwise_mean'``, ``'sum'`` or ``'none'``/``None``."""
    if reduction == "elementwise_mean":
        return torch.mean(x)
    if reduction == "none" or reduction is None:
        return x
    if reduction == "sum":
        return torch.sum(x)
    raise ValueError("Reduction parameter unknown.")


def class_reduce(num: Tensor, denom: Tensor, weights: Tensor, class_reduction: Optional[str] = "none") -> Tensor:
    """Reduce ``num / denom`` per class by micro / macro / weighted / none (NaNs from 0/0 become 0)."""
    valid = ("micro", "macro", "weighted", "none", None)
    frac = torch.sum(num) / torch.sum(denom) if class_reduction == "micro" else num / denom
    frac = torch.where(torch.isnan(frac), torch.zeros_like(frac), frac)
    if class_reduction == "micro":
        return frac
    if class_reduction == "macro":
        return torch.mean(frac)
    if class_reduction == "weighted":
        return torch.sum(frac * (weights.float() / torch.sum(weights)))
    if class_reduction == "none" or class_reduction is None:
        return frac
    raise ValueError(f"Reduction parameter {class_reduction} unknown. Choose between one of these: {valid}")


def _simple_gather_all_tensors(result: Tensor, group: Any, world_size: int) -> List[Tensor]:
    out = [torch.zeros_like(result) for _ in range(world_size)]
    torch.distributed.all_gather(out, result, group)
    return out


def gather_all_tensors(result: Tensor, group: Optional[Any] = None) -> List[Tensor]:
    """Gather ``result`` from every rank of ``group``; tensors may differ in shape across ranks.

    Returns a list with one tensor per rank (in rank order), each with its original shape.
    """
    if group is None:
        group = torch.distributed.group.WORLD
    result = result.contiguous()
    world_size = torch.distributed.get_world_size(group)
    torch.distributed.barrier(group=group)
    if result.ndim == 0:
        return _simple_gather_all_tensors(result, group, world_size)
    local_size = torch.tensor(result.shape, device=result.device)
    sizes = [torch.zeros_like(local_size) for _ in range(world_size)]
    torch.distributed.all_gather(sizes, local_size, group=group)
    stacked = torch.stack(sizes)
    max_size = stacked.max(dim=0).values
    if bool((stacked == max_size).all()):
        return _simple_gather_all_tensors(result, group, world_size)
    pad = []
    for dim_pad in reversed((max_size - local_size).cpu().tolist()):
        pad.extend([0, int(dim_pad)])
    padded = F.pad(result, pad)
    gathered = [torch.zeros_like(padded) for _ in range(world_size)]
    torch.distributed.all_gather(gathered, padded, group)
    for i, sz in enumerate(sizes):
        gathered[i] = gathered[i][tuple(slice(0, int(d)) for d in sz)]
    return gathered


__all__ = ["reduce", "class_reduce", "gather_all_tensors"]
