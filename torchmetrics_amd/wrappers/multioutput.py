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
    """Rows (dim 0) with a NaN anywhere in any of ``tensors``."""
    if not tensors:
        raise ValueError("Must pass at least one tensor as argument")
    rows = [torch.isnan(t.flatten(start_dim=1)).any(1) for t in tensors]
    return torch.stack(rows).any(0) if len(rows) > 1 else rows[0]


def _nan_rows_per_output(t: Tensor, output_dim: int, n_out: int) -> Tensor:
    """``[N, n_out]``: row r has a NaN in output slice i of ``t`` (all slices in one pass)."""
    per = torch.isnan(t).movedim(output_dim, -1)
    return per.reshape(per.shape[0], -1, n_out).any(1)


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
        n_out = len(self.metrics)
        drop = None
        if self.remove_nans:
            tensors = [t for t in (*args, *kwargs.values()) if isinstance(t, Tensor)]
            dim_ok = all(t.ndim >= 2 and self.output_dim % t.ndim != 0 and t.shape[self.output_dim] == n_out
                         for t in tensors)
            if tensors and dim_ok:
                # NaN rows of every output slice in one pass, and ONE host read: batches without NaNs (the common
                # case) skip the per-output boolean indexing and its device syncs altogether
                drop = torch.stack([_nan_rows_per_output(t, self.output_dim, n_out) for t in tensors]).any(0)
                if not bool(drop.any()):
                    drop = False
        out = []
        for i in range(n_out):
            sel = lambda t: t.narrow(self.output_dim, i, 1)  # noqa: E731  (view, no index tensor / copy)
            selected_args = apply_to_collection(args, Tensor, sel)
            selected_kwargs = apply_to_collection(kwargs, Tensor, sel)
            if self.remove_nans and drop is not False:
                keep = ~drop[:, i] if drop is not None else \
                    ~_get_nan_indices(*(tuple(selected_args) + tuple(selected_kwargs.values())))
                selected_args = [arg[keep] for arg in selected_args]
                selected_kwargs = {k: v[keep] for k, v in selected_kwargs.items()}
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
