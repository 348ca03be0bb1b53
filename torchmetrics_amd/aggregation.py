"""Streaming aggregators (parity: reference ``S/aggregation.py:30-727``).

NaN handling (``nan_strategy``) keeps the reference semantics, but on GPU tensors it avoids the reference's
``if nans.any()`` host sync (``S/aggregation.py:90``) wherever the result does not need the host:

* ``'error'``  -> a device-side flag (raised at ``compute()``, or per update with ``TORCHMETRICS_AMD_STRICT=1``);
* ``'ignore'`` / float -> NaNs are masked to the aggregator's neutral element / imputed in place, no sync;
* ``'warn'``   -> CPU: warns in ``update`` (a host check, as the reference).  ROCm: the NaNs are dropped on the device
  and a warning bit is raised in the validation word; the reference's UserWarning is emitted by the next
  ``compute()`` (``forward`` included), so the per-update host sync is gone.

On ROCm, Sum / Mean / Max / Min updates are one launch of ``csrc/common/aggregate.hip`` (NaN strategy, fp64
reduction and the in-place state fold together).
"""
from typing import Any, Callable, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops as _ops
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils import validation as _validation
from torchmetrics_amd.wrappers.running import Running


class BaseAggregator(Metric):
    """Base class for aggregators.

    Args:
        fn: reduction used for distributed sync (``"sum"``, ``"max"``, ...).
        default_value: default of the state.
        nan_strategy: ``'error'`` | ``'warn'`` | ``'ignore'`` | a float to impute.
        state_name: name of the state.
    """

    is_differentiable = None
    higher_is_better = None
    full_state_update: bool = False
    _neutral: float = 0.0  # value a masked-out NaN takes in the reduction (sum/mean: 0, max: -inf, min: +inf)

    def __init__(
        self,
        fn: Union[Callable, str],
        default_value: Union[Tensor, List],
        nan_strategy: Union[str, float] = "error",
        state_name: str = "value",
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        allowed = ("error", "warn", "ignore")
        if nan_strategy not in allowed and not isinstance(nan_strategy, float):
            raise ValueError(
                f"Arg `nan_strategy` should either be a float or one of {allowed} but got {nan_strategy}."
            )
        self.nan_strategy = nan_strategy
        self.add_state(state_name, default=default_value, dist_reduce_fx=fn)
        self.state_name = state_name

    def _cast_and_nan_check_input(
        self, x: Union[float, Tensor], weight: Optional[Union[float, Tensor]] = None, drop: bool = True
    ) -> Tuple[Tensor, Tensor]:
        """Cast to tensors of ``self.dtype`` and apply ``nan_strategy``.

        ``drop=False`` lets reduce-type aggregators replace NaNs by the neutral element instead of dropping them,
        which keeps shapes static (no host sync, HIP-graph capturable).
        """
        if not isinstance(x, Tensor):
            x = torch.as_tensor(x, dtype=self.dtype, device=self.device)
        if weight is not None and not isinstance(weight, Tensor):
            weight = torch.as_tensor(weight, dtype=self.dtype, device=self.device)
        if weight is None:
            weight = torch.ones_like(x)
            nan_mask = torch.isnan(x)
        else:
            nan_mask = torch.isnan(x) | torch.isnan(weight)
        strategy = self.nan_strategy
        if x.is_cuda and strategy == "error":
            flag = self._device_error_buffer(x.device)
            flag.bitwise_or_(nan_mask.any().to(torch.int32) * _validation.VALUE_NAN)
            return x.to(self.dtype), weight.to(self.dtype)
        if x.is_cuda and strategy == "ignore" and not drop:
            x = torch.where(nan_mask, torch.full_like(x, self._neutral), x)
            weight = torch.where(nan_mask, torch.zeros_like(weight), weight)
            return x.to(self.dtype), weight.to(self.dtype)
        if isinstance(strategy, float):
            x = torch.where(nan_mask, torch.full_like(x, strategy), x)
            weight = torch.where(nan_mask, torch.full_like(weight, strategy), weight)
            return x.to(self.dtype), weight.to(self.dtype)
        if bool(nan_mask.any()):
            if strategy == "error":
                raise RuntimeError("Encountered `nan` values in tensor")
            if strategy == "warn":
                rank_zero_warn("Encountered `nan` values in tensor. Will be removed.", UserWarning)
            keep = ~nan_mask
            x, weight = x[keep], weight[keep]
        return x.to(self.dtype), weight.to(self.dtype)

    def _fused_update(self, kind: int, value: Union[float, Tensor], weight: Union[float, Tensor, None],
                      s1: Optional[Tensor] = None) -> bool:
        """ROCm path: the whole update as one ``agg_update`` launch.  False when it does not apply (CPU states,
        autograd through the value, a state dtype other than f32 / f64): the caller runs the torch path."""
        s0 = getattr(self, self.state_name)
        if not (isinstance(s0, Tensor) and s0.is_cuda and s0.dtype in (torch.float32, torch.float64)):
            return False
        if isinstance(value, Tensor):
            if value.device != s0.device or (value.requires_grad and torch.is_grad_enabled()):
                return False
        else:
            value = torch.as_tensor(value, dtype=s0.dtype, device=s0.device)
        if value.dtype not in (torch.float32, torch.float64, torch.float16, torch.bfloat16):
            value = value.to(s0.dtype)
        if isinstance(weight, Tensor):
            if weight.device != s0.device or (weight.requires_grad and torch.is_grad_enabled()):
                return False
            if weight.numel() != 1:
                weight = torch.broadcast_to(weight, value.shape)
            if weight.dtype not in (torch.float32, torch.float64, torch.float16, torch.bfloat16):
                weight = weight.to(s0.dtype)
        if value.numel() == 0:
            return True
        strategy = self.nan_strategy
        if isinstance(strategy, float):
            mode, impute = _ops.AGG_NAN_IMPUTE, strategy
        else:
            modes = {"error": _ops.AGG_NAN_ERROR, "warn": _ops.AGG_NAN_WARN}
            mode, impute = modes.get(strategy, _ops.AGG_NAN_IGNORE), 0.0
        _ops.agg_update(value, weight, kind, mode, impute, self.__dict__, s0, s1, self._device_error_buffer(s0.device))
        return True

    def update(self, value: Union[float, Tensor]) -> None:
        """Overridden by subclasses."""

    def compute(self) -> Tensor:
        return getattr(self, self.state_name)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MaxMetric(BaseAggregator):
    """Running maximum."""

    full_state_update: bool = True
    max_value: Tensor
    _neutral = float("-inf")

    def __init__(self, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__("max", -torch.tensor(float("inf"), dtype=torch.get_default_dtype()), nan_strategy,
                         state_name="max_value", **kwargs)

    def update(self, value: Union[float, Tensor]) -> None:
        if self._fused_update(_ops.AGG_MAX, value, None):
            return
        value, _ = self._cast_and_nan_check_input(value, drop=False)
        if value.numel():
            self.max_value = torch.max(self.max_value, torch.max(value))


class MinMetric(BaseAggregator):
    """Running minimum."""

    full_state_update: bool = True
    min_value: Tensor
    _neutral = float("inf")

    def __init__(self, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__("min", torch.tensor(float("inf"), dtype=torch.get_default_dtype()), nan_strategy,
                         state_name="min_value", **kwargs)

    def update(self, value: Union[float, Tensor]) -> None:
        if self._fused_update(_ops.AGG_MIN, value, None):
            return
        value, _ = self._cast_and_nan_check_input(value, drop=False)
        if value.numel():
            self.min_value = torch.min(self.min_value, torch.min(value))


class SumMetric(BaseAggregator):
    """Running sum."""

    sum_value: Tensor

    def __init__(self, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__("sum", torch.tensor(0.0, dtype=torch.get_default_dtype()), nan_strategy,
                         state_name="sum_value", **kwargs)

    def update(self, value: Union[float, Tensor]) -> None:
        if self._fused_update(_ops.AGG_SUM, value, None):
            return
        value, _ = self._cast_and_nan_check_input(value, drop=False)
        if value.numel():
            self.sum_value += value.sum()


class CatMetric(BaseAggregator):
    """Concatenate every value seen."""

    _fold_cat_lists = True  # compute() only concatenates the list states

    value: Tensor

    def __init__(self, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__("cat", [], nan_strategy, **kwargs)

    def update(self, value: Union[float, Tensor]) -> None:
        value, _ = self._cast_and_nan_check_input(value)
        if value.numel():
            self.value.append(value)

    def compute(self) -> Tensor:
        if isinstance(self.value, list) and self.value:
            return dim_zero_cat(self.value)
        return self.value


class MeanMetric(BaseAggregator):
    """Running (weighted) mean."""

    mean_value: Tensor

    def __init__(self, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__("sum", torch.tensor(0.0, dtype=torch.get_default_dtype()), nan_strategy,
                         state_name="mean_value", **kwargs)
        self.add_state("weight", default=torch.tensor(0.0, dtype=torch.get_default_dtype()), dist_reduce_fx="sum")

    def update(self, value: Union[float, Tensor], weight: Union[float, Tensor] = 1.0) -> None:
        if self._fused_update(_ops.AGG_MEAN, value, weight, self.weight):
            return
        if not isinstance(value, Tensor):
            value = torch.as_tensor(value, dtype=self.dtype, device=self.device)
        if weight is not None and not isinstance(weight, Tensor):
            weight = torch.as_tensor(weight, dtype=self.dtype, device=self.device)
        weight = torch.broadcast_to(weight, value.shape)
        value, weight = self._cast_and_nan_check_input(value, weight, drop=False)
        if value.numel() == 0:
            return
        self.mean_value += (value * weight).sum()
        self.weight += weight.sum()

    def compute(self) -> Tensor:
        return self.mean_value / self.weight


class RunningMean(Running):
    """Mean over a sliding window of the last ``window`` updates."""

    def __init__(self, window: int = 5, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__(base_metric=MeanMetric(nan_strategy=nan_strategy, **kwargs), window=window)


class RunningSum(Running):
    """Sum over a sliding window of the last ``window`` updates."""

    def __init__(self, window: int = 5, nan_strategy: Union[str, float] = "warn", **kwargs: Any) -> None:
        super().__init__(base_metric=SumMetric(nan_strategy=nan_strategy, **kwargs), window=window)


__all__ = ["CatMetric", "MaxMetric", "MeanMetric", "MinMetric", "RunningMean", "RunningSum", "SumMetric"]
