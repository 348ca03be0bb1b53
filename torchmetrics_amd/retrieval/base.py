"""Retrieval module base (parity: reference ``S/retrieval/base.py:26-190``).

States are the reference's three ``cat`` lists (``indexes``, ``preds``, ``target``; ``dist_reduce_fx=None`` so a
DDP sync gathers them).  ``compute`` evaluates every query in one segmented pass
(:mod:`torchmetrics_amd.functional.retrieval._segments`); subclasses that only implement the reference's per-query
``_metric`` hook still work through the per-query fallback loop.
"""
from abc import ABC
from typing import Any, Callable, List, Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.retrieval._segments import Segments
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.checks import _check_retrieval_inputs
from torchmetrics_amd.utilities.data import dim_zero_cat


def _retrieval_aggregate(
    values: Tensor,
    aggregation: Union[Literal["mean", "median", "min", "max"], Callable] = "mean",
    dim: Optional[int] = None,
) -> Tensor:
    if aggregation == "mean":
        return values.mean() if dim is None else values.mean(dim=dim)
    if aggregation == "median":
        return values.median() if dim is None else values.median(dim=dim).values
    if aggregation == "min":
        return values.min() if dim is None else values.min(dim=dim).values
    if aggregation == "max":
        return values.max() if dim is None else values.max(dim=dim).values
    return aggregation(values, dim=dim)


def _aggregate_queries(vals: Tensor, empty: Tensor, nq: Tensor, action: str, aggregation, like: Tensor,
                       error_msg: str) -> Tensor:
    """Empty-query policy + aggregation of per-query values on the device (``mean``: no host read at all)."""
    valid = torch.arange(vals.numel(), device=vals.device) < nq.to(vals.device)
    empty = empty.bool() & valid
    if action == "error" and bool(empty.any()):
        raise ValueError(error_msg)
    if action == "pos":
        vals = torch.where(empty, torch.ones_like(vals), vals)
    elif action == "neg":
        vals = torch.where(empty, torch.zeros_like(vals), vals)
    else:
        valid = valid & ~empty
    if aggregation == "mean":
        cnt = valid.sum()
        mean = torch.where(valid, vals, torch.zeros_like(vals)).sum() / cnt.clamp(min=1)
        return torch.where(cnt > 0, mean, torch.zeros_like(mean)).to(like)
    sel = vals[valid]
    if sel.numel() == 0:
        return torch.tensor(0.0).to(like)
    return _retrieval_aggregate(sel.to(like), aggregation)


class RetrievalMetric(Metric, ABC):
    """Base for query-grouped metrics: ``update(preds, target, indexes)``; ``indexes`` names each doc's query."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    indexes: List[Tensor]
    preds: List[Tensor]
    target: List[Tensor]

    def __init__(
        self,
        empty_target_action: str = "neg",
        ignore_index: Optional[int] = None,
        aggregation: Union[Literal["mean", "median", "min", "max"], Callable] = "mean",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        self.allow_non_binary_target = False
        if empty_target_action not in ("error", "skip", "neg", "pos"):
            raise ValueError(f"Argument `empty_target_action` received a wrong value `{empty_target_action}`.")
        self.empty_target_action = empty_target_action
        if ignore_index is not None and not isinstance(ignore_index, int):
            raise ValueError("Argument `ignore_index` must be an integer or None.")
        self.ignore_index = ignore_index
        if not (aggregation in ("mean", "median", "min", "max") or callable(aggregation)):
            raise ValueError(
                "Argument `aggregation` must be one of `mean`, `median`, `min`, `max` or a custom callable function"
                f"which takes tensor of values, but got {aggregation}."
            )
        self.aggregation = aggregation
        self.add_state("indexes", default=[], dist_reduce_fx=None)
        self.add_state("preds", default=[], dist_reduce_fx=None)
        self.add_state("target", default=[], dist_reduce_fx=None)

    def update(self, preds: Tensor, target: Tensor, indexes: Tensor) -> None:
        if indexes is None:
            raise ValueError("Argument `indexes` cannot be None")
        indexes, preds, target = _check_retrieval_inputs(
            indexes, preds, target, allow_non_binary_target=self.allow_non_binary_target, ignore_index=self.ignore_index
        )
        self.indexes.append(indexes)
        self.preds.append(preds)
        self.target.append(target)

    # -- hooks -------------------------------------------------------------------------------------------------
    def _kernel_kind(self) -> Optional[Tuple[str, Optional[int], bool]]:
        """``(kind, top_k, adaptive_k)`` of :func:`torchmetrics_amd.ops.retrieval_metric`, or ``None``."""
        return None

    def _segment_metric(self, seg: Segments) -> Optional[Tensor]:
        """Per-query scores for all queries at once; ``None`` -> per-query ``_metric`` fallback."""
        return None

    def _metric(self, preds: Tensor, target: Tensor) -> Tensor:
        raise NotImplementedError

    def _empty_queries(self, seg: Segments) -> Tensor:
        """Queries without any relevant document (fall-out overrides: without any non-relevant one)."""
        return seg.seg_sum(seg.target) == 0

    def _empty_error(self) -> str:
        return "`compute` method was provided with a query with no positive target."

    # -- compute -----------------------------------------------------------------------------------------------
    def compute(self) -> Tensor:
        preds = dim_zero_cat(self.preds)
        target = dim_zero_cat(self.target)
        spec = self._kernel_kind()
        if spec is not None and preds.is_cuda:
            vals, empty, nq = ops.retrieval_metric(preds, target, dim_zero_cat(self.indexes), *spec)
            return _aggregate_queries(vals, empty, nq, self.empty_target_action, self.aggregation, preds,
                                      self._empty_error())
        seg = Segments(preds, target, dim_zero_cat(self.indexes))
        if seg.num_groups == 0:
            return torch.tensor(0.0).to(preds)
        empty = self._empty_queries(seg)
        if self.empty_target_action == "error" and bool(empty.any()):
            raise ValueError(self._empty_error())
        scores = self._segment_metric(seg)
        if scores is None:
            scores = self._per_query(seg, empty)
        if self.empty_target_action == "pos":
            scores = torch.where(empty, torch.ones_like(scores), scores)
        elif self.empty_target_action == "neg":
            scores = torch.where(empty, torch.zeros_like(scores), scores)
        else:  # skip
            scores = scores[~empty]
        if scores.numel() == 0:
            return torch.tensor(0.0).to(preds)
        return _retrieval_aggregate(scores.to(preds), self.aggregation)

    def _per_query(self, seg: Segments, empty: Tensor) -> Tensor:
        sizes = seg.size.tolist()
        skip = empty.tolist()
        out = [0.0 if e else self._metric(p, t)
               for p, t, e in zip(seg.preds.split(sizes), seg.target.split(sizes), skip)]
        return torch.stack([torch.as_tensor(x, dtype=torch.float32, device=seg.preds.device) for x in out])
