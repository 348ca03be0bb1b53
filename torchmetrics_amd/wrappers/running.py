"""Sliding-window wrapper (parity: reference ``S/wrappers/running.py:27-133``).

The window keeps ``window`` snapshots of the wrapped metric's *batch* states (slot ``i`` registered as
``<state>_<i>``); ``compute`` folds them with the wrapped metric's own ``_reduce_states`` so any metric with
``full_state_update=False`` works unchanged.
"""
from typing import Any, Optional, Sequence, Union

import torch
from torch import Tensor

from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_max, dim_zero_min, dim_zero_sum
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_amd.wrappers.abstract import WrapperMetric


_WINDOW_FOLDS = {
    dim_zero_sum: torch.sum,
    dim_zero_max: lambda x, d: torch.amax(x, d),
    dim_zero_min: lambda x, d: torch.amin(x, d),
}


class Running(WrapperMetric):
    """Compute ``base_metric`` over the last ``window`` updates only."""

    def __init__(self, base_metric: Metric, window: int = 5) -> None:
        super().__init__()
        if not isinstance(base_metric, Metric):
            raise ValueError(
                f"Expected argument `metric` to be an instance of `torchmetrics.Metric` but got {base_metric}"
            )
        if not (isinstance(window, int) and window > 0):
            raise ValueError(f"Expected argument `window` to be a positive integer but got {window}")
        self.base_metric = base_metric
        self.window = window
        if base_metric.full_state_update is not False:
            raise ValueError(
                f"Expected attribute `full_state_update` set to `False` but got {base_metric.full_state_update}"
            )
        self._num_vals_seen = 0
        for key in base_metric._defaults:
            for slot in range(window):
                self.add_state(
                    name=f"{key}_{slot}", default=base_metric._defaults[key], dist_reduce_fx=base_metric._reductions[key]
                )

    def _store_slot(self) -> None:
        slot = self._num_vals_seen % self.window
        for key in self.base_metric._defaults:
            setattr(self, f"{key}_{slot}", getattr(self.base_metric, key))
        self.base_metric.reset()
        self._num_vals_seen += 1

    def update(self, *args: Any, **kwargs: Any) -> None:
        self.base_metric.update(*args, **kwargs)
        self._store_slot()

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        res = self.base_metric.forward(*args, **kwargs)
        self._store_slot()
        self._computed = None
        return res

    def compute(self) -> Any:
        base = self.base_metric
        for key in base._defaults:
            slots = [getattr(self, f"{key}_{i}") for i in range(self.window)]
            fold = _WINDOW_FOLDS.get(base._reductions[key])
            if fold is not None and all(isinstance(t, Tensor) for t in slots):
                # the whole window in one reduction over the stacked slots (sum / max / min states)
                setattr(base, key, fold(torch.stack([getattr(base, key), *slots]), 0))
            else:
                for t in slots:  # order-dependent reductions: the wrapped metric's own pairwise merge
                    base._reduce_states({k: (t if k == key else getattr(base, k)) for k in base._defaults},
                                        only=key)
        base._update_count = self._num_vals_seen
        val = base.compute()
        base.reset()
        return val

    def reset(self) -> None:
        super().reset()
        self._num_vals_seen = 0

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
