"""Bootstrapped confidence statistics of any metric (reference ``S/wrappers/bootstrapping.py:25-190``)."""
from copy import deepcopy
from typing import Any, Dict, Optional, Union

import torch
from torch import Tensor
from torch.nn import ModuleList

from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import apply_to_collection
from torchmetrics_amd.wrappers.abstract import WrapperMetric


def _bootstrap_sampler(size: int, sampling_strategy: str = "poisson") -> Tensor:
    """Resampling indices: Poisson(1) multiplicities (``repeat_interleave``) or multinomial with replacement.

    Drawn with the global CPU generator like the reference, so seeded runs resample identically.
    """
    if sampling_strategy == "poisson":
        n = torch.distributions.Poisson(1).sample((size,))
        return torch.arange(size).repeat_interleave(n.long(), dim=0)
    if sampling_strategy == "multinomial":
        return torch.multinomial(torch.ones(size), num_samples=size, replacement=True)
    raise ValueError("Unknown sampling strategy")


class BootStrapper(WrapperMetric):
    """Keeps ``num_bootstraps`` copies of ``base_metric``, each updated on a resampled batch.

    ``compute`` returns a dict with the mean / std / quantile / raw values over the copies.
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
        self.metrics = ModuleList([deepcopy(base_metric) for _ in range(num_bootstraps)])
        self.num_bootstraps = num_bootstraps
        self.mean = mean
        self.std = std
        self.quantile = quantile
        self.raw = raw
        allowed_sampling = ("poisson", "multinomial")
        if sampling_strategy not in allowed_sampling:
            raise ValueError(
                f"Expected argument ``sampling_strategy`` to be one of {allowed_sampling}"
                f" but received {sampling_strategy}"
            )
        self.sampling_strategy = sampling_strategy

    def update(self, *args: Any, **kwargs: Any) -> None:
        args_sizes = apply_to_collection(args, Tensor, len)
        kwargs_sizes = list(apply_to_collection(kwargs, Tensor, len))
        if len(args_sizes) > 0:
            size = args_sizes[0]
        elif len(kwargs_sizes) > 0:
            size = kwargs_sizes[0]
        else:
            raise ValueError("None of the input contained tensors, so could not determine the sampling size")
        for idx in range(self.num_bootstraps):
            sample_idx = _bootstrap_sampler(size, sampling_strategy=self.sampling_strategy).to(self.device,
                                                                                                 non_blocking=True)
            if sample_idx.numel() == 0:
                continue
            new_args = apply_to_collection(args, Tensor, torch.index_select, dim=0, index=sample_idx)
            new_kwargs = apply_to_collection(kwargs, Tensor, torch.index_select, dim=0, index=sample_idx)
            self.metrics[idx].update(*new_args, **new_kwargs)

    def compute(self) -> Dict[str, Tensor]:
        computed_vals = torch.stack([m.compute() for m in self.metrics], dim=0)
        out = {}
        if self.mean:
            out["mean"] = computed_vals.mean(dim=0)
        if self.std:
            out["std"] = computed_vals.std(dim=0)
        if self.quantile is not None:
            out["quantile"] = torch.quantile(computed_vals, self.quantile)
        if self.raw:
            out["raw"] = computed_vals
        return out

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return super(WrapperMetric, self).forward(*args, **kwargs)
