"""Segmented (per-query) retrieval engine.

The reference computes retrieval metrics by sorting on the query index, copying the group sizes to the host and
looping over queries in Python (``S/retrieval/base.py:147-190``), one tiny ``topk``/``argsort`` per query.  Here all
queries are processed at once: two stable device sorts order the documents by (query, score descending), and every
metric becomes a segmented reduction over that order (``index_add`` / ``scatter_reduce`` / segmented ``cumsum``).
The only host synchronisation is reading the number of queries.
"""
from typing import Optional

import torch
from torch import Tensor


class Segments:
    """Documents sorted by (query, score desc) with per-document rank and per-query statistics."""

    def __init__(self, preds: Tensor, target: Tensor, indexes: Optional[Tensor] = None) -> None:
        dev = preds.device
        order = torch.argsort(preds, descending=True, stable=True)
        if indexes is not None:
            order = order[torch.argsort(indexes[order], stable=True)]
            idx = indexes[order]
        else:
            idx = torch.zeros(preds.numel(), dtype=torch.long, device=dev)
        self.preds = preds[order]
        self.target = target[order]
        self.query = idx
        n = preds.numel()
        start = torch.ones(n, dtype=torch.bool, device=dev)
        if n > 1:
            start[1:] = idx[1:] != idx[:-1]
        self.is_start = start
        self.gid = torch.cumsum(start.long(), 0) - 1
        self.num_groups = int(self.gid[-1].item()) + 1 if n else 0
        self.starts = torch.nonzero(start).flatten()
        self.pos = torch.arange(n, device=dev) - self.starts[self.gid]
        self.size = torch.bincount(self.gid, minlength=self.num_groups)

    # ---------------------------------------------------------------------------------------------- primitives
    def seg_sum(self, x: Tensor) -> Tensor:
        out = torch.zeros(self.num_groups, dtype=torch.float64 if x.is_floating_point() else torch.long,
                          device=x.device)
        return out.index_add_(0, self.gid, x.to(out.dtype))

    def seg_cumsum(self, x: Tensor) -> Tensor:
        cs = torch.cumsum(x.to(torch.float64), 0)
        base = torch.where(self.starts > 0, cs[(self.starts - 1).clamp(min=0)], torch.zeros_like(cs[self.starts]))
        return cs - base[self.gid]

    def seg_min(self, x: Tensor, fill: float) -> Tensor:
        out = torch.full((self.num_groups,), fill, dtype=x.dtype, device=x.device)
        return out.scatter_reduce_(0, self.gid, x, reduce="amin", include_self=True)

    def k_per_group(self, top_k: Optional[int]) -> Tensor:
        return self.size if top_k is None else torch.full_like(self.size, top_k)

    def in_top(self, k_g: Tensor) -> Tensor:
        return self.pos < k_g[self.gid]

    def tie_groups(self) -> Tensor:
        """Start flags of runs of equal scores inside each query."""
        tie_start = self.is_start.clone()
        if self.preds.numel() > 1:
            tie_start[1:] |= self.preds[1:] != self.preds[:-1]
        return tie_start
