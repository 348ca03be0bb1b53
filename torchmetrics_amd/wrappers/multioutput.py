"""Apply a metric independently along an output dimension (reference ``S/wrappers/multioutput.py:27-180``)."""
from copy import deepcopy
from typing import Any, List, Tuple

import torch
from torch import Tensor
from torch.nn import ModuleList

from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import apply_to_collection
from torchmetrics_amd.wrappers.abstract import WrapperMetric


def _get_nan_indices(*tensors: Tensor) -> Tensor:
    if len(tensors) == 0:
        raise ValueError("Must pass at least one tensor as argument")
    nan_idxs = torch.zeros(len(tensors[0]), dtype=torch.bool, device=tensors[0].device)
    for t in tensors:
        nan_idxs |= torch.any(torch.isnan(t.flatten(start_dim=1)), dim=1)
    return nan_idxs


class MultioutputWrapper(WrapperMetric):
    """One copy of ``base_metric`` per output slice along ``output_dim`` (rows with NaNs optionally dropped)."""

    is_differentiable = False

    def __init__(
        self,
        base_metric: Metric,
        num_outputs: int,
        output_dim: int = -1,
        remove_nans: bool = True,
        squeeze_outputs: bool = True,
    ) -> None:
        super().__init__()
        self.metrics = ModuleList([deepcopy(base_metric) for _ in range(num_outputs)])
        self.output_dim = output_dim
        self.remove_nans = remove_nans
        self.squeeze_outputs = squeeze_outputs

    def _get_args_kwargs_by_output(self, *args: Tensor, **kwargs: Tensor) -> List[Tuple[Any, Any]]:
        out = []
        for i in range(len(self.metrics)):
            sel = lambda t: t.narrow(self.output_dim, i, 1)  # noqa: E731  (view, no index tensor / copy)
            selected_args = apply_to_collection(args, Tensor, sel)
            selected_kwargs = apply_to_collection(kwargs, Tensor, sel)
            if self.remove_nans:
                nan_idxs = _get_nan_indices(*(tuple(selected_args) + tuple(selected_kwargs.values())))
                selected_args = [arg[~nan_idxs] for arg in selected_args]
                selected_kwargs = {k: v[~nan_idxs] for k, v in selected_kwargs.items()}
            if self.squeeze_outputs:
                selected_args = [arg.squeeze(self.output_dim) for arg in selected_args]
                selected_kwargs = {k: v.squeeze(self.output_dim) for k, v in selected_kwargs.items()}
            out.append((selected_args, selected_kwargs))
        return out

    def update(self, *args: Any, **kwargs: Any) -> None:
        for metric, (a, k) in zip(self.metrics, self._get_args_kwargs_by_output(*args, **kwargs)):
            metric.update(*a, **k)

    def compute(self) -> Tensor:
        return torch.stack([m.compute() for m in self.metrics], 0)

    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        results = [metric(*a, **k) for metric, (a, k) in zip(self.metrics, self._get_args_kwargs_by_output(*args,
                                                                                                            **kwargs))]
        if results[0] is None:
            return None
        return torch.stack(results, 0)

    def reset(self) -> None:
        for metric in self.metrics:
            metric.reset()
        super().reset()
