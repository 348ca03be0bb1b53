"""Running extrema of a scalar metric over its ``compute`` calls (reference ``S/wrappers/minmax.py:25-140``).

The extrema live in one 2-element tensor ``[min, max]`` on the wrapped metric's device and are folded with one
``torch.stack`` + ``aminmax``-style select per ``compute()``: no host round trip, whatever the value's device.
"""
from typing import Any, Dict, Optional, Union

import torch
from torch import Tensor

from torchmetrics_amd.metric import Metric
from torchmetrics_amd.wrappers.abstract import WrapperMetric


def _scalar_like(val: Any) -> bool:
    return isinstance(val, (int, float)) or (isinstance(val, Tensor) and val.numel() == 1)


class MinMaxMetric(WrapperMetric):
    """``compute`` returns ``{"raw", "max", "min"}`` of the wrapped scalar metric."""

    full_state_update: Optional[bool] = True

    def __init__(self, base_metric: Metric, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(base_metric, Metric):
            raise ValueError(
                f"Expected base metric to be an instance of `torchmetrics.Metric` but received {base_metric}"
            )
        self._base_metric = base_metric
        self._extrema = torch.tensor([float("inf"), float("-inf")])

    # the reference exposes the two running values as attributes
    @property
    def min_val(self) -> Tensor:
        return self._extrema[0]

    @min_val.setter
    def min_val(self, value: Union[float, Tensor]) -> None:
        self._extrema = torch.stack([torch.as_tensor(value, dtype=self._extrema.dtype).to(self._extrema.device),
                                     self._extrema[1]])

    @property
    def max_val(self) -> Tensor:
        return self._extrema[1]

    @max_val.setter
    def max_val(self, value: Union[float, Tensor]) -> None:
        self._extrema = torch.stack([self._extrema[0],
                                     torch.as_tensor(value, dtype=self._extrema.dtype).to(self._extrema.device)])

    def update(self, *args: Any, **kwargs: Any) -> None:
        self._base_metric.update(*args, **kwargs)

    def compute(self) -> Dict[str, Tensor]:
        raw = self._base_metric.compute()
        if not _scalar_like(raw):
            raise RuntimeError(f"Returned value from base metric should be a float or scalar tensor, but got {raw}.")
        raw = torch.as_tensor(raw)
        dt = torch.promote_types(self._extrema.dtype, raw.dtype) if raw.is_floating_point() else self._extrema.dtype
        ext = self._extrema.to(device=raw.device, dtype=dt)
        v = raw.reshape(()).to(dt)
        # NaN-propagating like the reference's comparisons: a NaN value never replaces an extremum
        lo = torch.where(ext[0] > v, v, ext[0])
        hi = torch.where(ext[1] < v, v, ext[1])
        self._extrema = torch.stack([lo, hi])
        return {"raw": raw, "max": self._extrema[1], "min": self._extrema[0]}

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return super(WrapperMetric, self).forward(*args, **kwargs)

    def reset(self) -> None:
        super().reset()
        self._base_metric.reset()

    @staticmethod
    def _is_suitable_val(val: Union[float, Tensor]) -> bool:
        return _scalar_like(val)
