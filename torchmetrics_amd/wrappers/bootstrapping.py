"""Bootstrapped confidence statistics of a metric (API of reference ``S/wrappers/bootstrapping.py:54-190``).

Resampling model.  A bootstrap replicate of a batch of ``n`` samples is a vector of multiplicities ``w[i] >= 0``:
Poisson(1) draws (``sampling_strategy="poisson"``) or the counts of ``n`` uniform draws with replacement
(``"multinomial"``).  The draws are made exactly as the reference makes them -- the global CPU generator, one draw
per replicate, in replicate order -- so a seeded run sees the same replicates and reproduces the reference's
statistics; only the multiplicities (``B x n`` small integers) then travel to the device, in ONE copy.

Update paths.

* **Batched** (multiclass stat-score family -- accuracy, precision, recall, F-beta, specificity, Hamming, stat
  scores -- with ``top_k=1`` and global averaging): the B replicates' states are stacked ``[B, C]`` tensors (each
  copy's state is a view of its row) and one kernel turns (preds, target, multiplicities) into the weighted
  per-replicate histograms (``csrc/classification/bootstrap.hip``), one more folds them into the states.  ``compute``
  evaluates all replicates in one fused reduction (the stacked states read as B "samples").
* **General** (any other metric): the replicates' sample indices are concatenated and every input tensor is gathered
  once for all replicates; each copy then updates on its slice.
"""
from copy import deepcopy
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import ModuleList

from torchmetrics_amd import ops
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import apply_to_collection
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_amd.wrappers.abstract import WrapperMetric

_STRATEGIES = ("poisson", "multinomial")


def _bootstrap_sampler(size: int, sampling_strategy: str = "poisson") -> Tensor:
    """Sample indices of one replicate (sorted multiplicities for Poisson, draw order for multinomial)."""
    if sampling_strategy == "poisson":
        counts = torch.distributions.Poisson(1).sample((size,)).long()
        return torch.repeat_interleave(torch.arange(size), counts)
    if sampling_strategy == "multinomial":
        return torch.multinomial(torch.ones(size), num_samples=size, replacement=True)
    raise ValueError("Unknown sampling strategy")


def _draw_replicates(size: int, reps: int, strategy: str) -> List[Tensor]:
    """``reps`` replicates' index vectors, drawn in the reference's order from the global CPU generator."""
    return [_bootstrap_sampler(size, strategy) for _ in range(reps)]


def _first_len(args: tuple, kwargs: dict) -> int:
    for coll in (args, tuple(kwargs.values())):
        sizes = apply_to_collection(coll, Tensor, len)
        flat = [s for s in (sizes if isinstance(sizes, (list, tuple)) else [sizes]) if isinstance(s, int)]
        if flat:
            return flat[0]
    raise ValueError("None of the input contained tensors, so could not determine the sampling size")


class _StackedStatScores:
    """Batched path for the multiclass stat-score family: stacked [B, C] states, one weighted-histogram kernel."""

    def __init__(self, copies: ModuleList) -> None:
        self.copies = copies
        self.template = deepcopy(copies[0])  # evaluates all replicates at once in compute()
        self.stacked: Optional[Tuple[Tensor, ...]] = None
        self.ws: Optional[Tensor] = None

    @staticmethod
    def supports(metric: Metric) -> bool:
        from torchmetrics_amd.classification.stat_scores import MulticlassStatScores

        return (isinstance(metric, MulticlassStatScores) and getattr(metric, "top_k", 1) == 1
                and metric.multidim_average == "global")

    def _bind(self, device: torch.device) -> Tuple[Tensor, ...]:
        """Stack the copies' states once and make every copy's state a view of its row (kept in sync by identity)."""
        names = ("tp", "fp", "tn", "fn")
        if self.stacked is not None and self.stacked[0].device == device and all(
                getattr(m, n)._base is s for m in self.copies for n, s in zip(names, self.stacked)):
            return self.stacked
        stacked = tuple(torch.stack([getattr(m, n).to(device) for m in self.copies]).contiguous() for n in names)
        for b, m in enumerate(self.copies):
            for n, s in zip(names, stacked):
                setattr(m, n, s[b])
        self.stacked = stacked
        return stacked

    def update(self, replicates: List[Tensor], preds: Tensor, target: Tensor) -> None:
        m0 = self.copies[0]
        if m0.validate_args:
            from torchmetrics_amd.functional.classification.stat_scores import (
                _multiclass_stat_scores_tensor_validation,
            )

            _multiclass_stat_scores_tensor_validation(preds, target, m0.num_classes, "global", m0.ignore_index)
        n = target.shape[0]
        dev = preds.device
        stacked = self._bind(dev)
        c = m0.num_classes
        reps = len(replicates)
        counts = torch.stack([torch.bincount(r, minlength=n) for r in replicates], dim=1).to(torch.int32)  # [n, B]
        weights = counts.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else counts
        if self.ws is None or self.ws.device != dev or self.ws.numel() != reps * (3 * c + 1):
            self.ws = torch.zeros(reps, 3 * c + 1, dtype=torch.int64, device=dev)
        flag = m0._device_error_buffer(dev)  # raised by compute() with the base metric's message
        p = preds if preds.is_floating_point() else preds.long()
        ops.mc_bootstrap_update(p.reshape(n, -1).contiguous() if p.is_floating_point() else p.reshape(n).contiguous(),
                                target.reshape(n).contiguous(), weights, self.ws, flag, c, m0.ignore_index)
        micro = stacked[0].shape[1] == 1 and c > 1
        ops.mc_stats_finalize(self.ws, c, micro, True, *stacked)
        if not preds.is_cuda:
            m0._raise_device_errors()
        for m in self.copies:
            m.__dict__["_update_count"] += 1
            m.__dict__["_computed"] = None

    def compute(self) -> Tensor:
        self.copies[0]._raise_device_errors()
        t = self.template
        for n, s in zip(("tp", "fp", "tn", "fn"), self.stacked):
            t.__dict__[n] = s
        t.__dict__["multidim_average"] = "samplewise"  # rows = replicates
        try:
            return type(t).compute(t)
        finally:
            t.__dict__["multidim_average"] = "global"


class BootStrapper(WrapperMetric):
    """Keep ``num_bootstraps`` replicates of ``base_metric``, each fed a resampling of every batch.

    ``compute`` returns a dict with the replicates' ``mean`` / ``std`` / ``quantile`` / ``raw`` values.
    """

    full_state_update: Optional[bool] = True

    def __init__(
        self,
        base_metric: Metric,
        num_bootstraps: int = 10,
        mean: bool = True,
        std: bool = True,
        quantile: Optional[Union[float, Tensor]] = None,
        raw: bool = False,
        sampling_strategy: str = "poisson",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if not isinstance(base_metric, Metric):
            raise ValueError(
                f"Expected base metric to be an instance of torchmetrics.Metric but received {base_metric}"
            )
        if sampling_strategy not in _STRATEGIES:
            raise ValueError(
                f"Expected argument ``sampling_strategy`` to be one of {_STRATEGIES}"
                f" but received {sampling_strategy}"
            )
        self.metrics = ModuleList(deepcopy(base_metric) for _ in range(num_bootstraps))
        self.num_bootstraps = num_bootstraps
        self.mean, self.std, self.quantile, self.raw = mean, std, quantile, raw
        self.sampling_strategy = sampling_strategy
        self._stacked = _StackedStatScores(self.metrics) if (
            num_bootstraps > 0 and _StackedStatScores.supports(base_metric)) else None

    # ------------------------------------------------------------------------------------------------ update
    def update(self, *args: Any, **kwargs: Any) -> None:
        size = _first_len(args, kwargs)
        replicates = _draw_replicates(size, self.num_bootstraps, self.sampling_strategy)
        if self._stacked is not None and not kwargs and len(args) == 2 and all(isinstance(a, Tensor) for a in args):
            self._stacked.update(replicates, *args)
            return
        self._gathered_update(replicates, args, kwargs)

    def _gathered_update(self, replicates: List[Tensor], args: tuple, kwargs: dict) -> None:
        """Every input gathered ONCE for all replicates (concatenated indices), then one update per replicate."""
        lengths = [r.numel() for r in replicates]
        if sum(lengths) == 0:
            return
        idx = torch.cat(replicates).to(self.device, non_blocking=True)
        big_args = apply_to_collection(args, Tensor, torch.index_select, dim=0, index=idx)
        big_kwargs = apply_to_collection(kwargs, Tensor, torch.index_select, dim=0, index=idx)
        start = 0
        for m, ln in zip(self.metrics, lengths):
            if ln:
                take = lambda x, s=start, e=start + ln: x[s:e]  # noqa: E731
                m.update(*apply_to_collection(big_args, Tensor, take), **apply_to_collection(big_kwargs, Tensor, take))
            start += ln

    # ----------------------------------------------------------------------------------------------- compute
    def _replicate_values(self) -> Tensor:
        if self._stacked is not None and self._stacked.stacked is not None:
            return self._stacked.compute()
        return torch.stack([m.compute() for m in self.metrics], dim=0)

    def compute(self) -> Dict[str, Tensor]:
        vals = self._replicate_values()
        stats: Dict[str, Tensor] = {}
        if self.mean:
            stats["mean"] = vals.mean(dim=0)
        if self.std:
            stats["std"] = vals.std(dim=0)
        if self.quantile is not None:
            stats["quantile"] = torch.quantile(vals, self.quantile)
        if self.raw:
            stats["raw"] = vals
        return stats

    def reset(self) -> None:
        super().reset()
        if self._stacked is not None:
            self._stacked.stacked = None  # the copies re-created their states

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return super(WrapperMetric, self).forward(*args, **kwargs)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None
             ) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
