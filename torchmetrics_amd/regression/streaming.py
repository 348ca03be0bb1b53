"""Streaming regression module metrics (sum states).

Parity: reference ``S/regression/{mse,mae,mape,symmetric_mape,wmape,log_mse,log_cosh,r2,rse,explained_variance,
minkowski,tweedie_deviance,csi}.py`` -- same constructor arguments, state names, dtypes and reductions.

``update`` is one call of the fused moments kernel that adds straight into the state tensors (``dests``), i.e. two
HIP launches per update whatever the number of states, no temporaries, no host syncs.
"""
from typing import Any, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor, tensor

from torchmetrics_amd import ops
from torchmetrics_amd.functional.regression.streaming import (
    EPS,
    _check_data_shape_to_num_outputs,
    _critical_success_index_compute,
    _critical_success_index_update,
    _explained_variance_compute,
    _log_cosh_error_compute,
    _mean_absolute_error_compute,
    _mean_absolute_percentage_error_compute,
    _mean_squared_error_compute,
    _mean_squared_log_error_compute,
    _minkowski_distance_compute,
    _r2_score_compute,
    _relative_squared_error_compute,
    _symmetric_mean_absolute_percentage_error_compute,
    _tweedie_deviance_score_compute,
    _tweedie_deviance_score_update,
    _weighted_mean_absolute_percentage_error_compute,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.data import dim_zero_cat
from torchmetrics_amd.utilities.exceptions import TorchMetricsUserError
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


_EV_IDS = [ops.sum_diff(ops.ST, ops.SP), ops.SSE, ops.ST, ops.STT, ops.COUNT]


class _MomentsMetric(Metric):
    """Base: subclasses declare ``_moments = [(state_name, sum_id), ...]`` and the kernel fills them in one pass."""

    _moments: List[Tuple[str, int]] = []
    _k: int = 1
    _eps: float = EPS
    _power: float = 2.0

    def _fused_update(self, preds: Tensor, target: Tensor, k: int = 1) -> None:
        d = self.__dict__
        dests = [getattr(self, name) for name, _ in self._moments]
        checked = preds.is_cuda and ops.states_ready(d, tuple(dests), preds.get_device())
        if not checked and not all(t.device == preds.device and t.is_contiguous() for t in dests):
            dests = [t.to(preds.device).contiguous() for t in dests]
            for (name, _), t in zip(self._moments, dests):
                setattr(self, name, t)
        ids = d.get("_moment_ids")
        if ids is None:
            ids = d["_moment_ids"] = [sid for _, sid in self._moments]
        self._submit(ops.MomentsPlan(preds.reshape(-1, k), target.reshape(-1, k), k, dests, ids, eps=self._eps,
                                     power=self._power, src=(preds, target), checked=checked))

    def _submit(self, plan: "ops.MomentsPlan") -> None:
        """Run the kernel now, or hand the plan to the enclosing ``MetricCollection.update``, which merges the plans
        of all its streaming regression members on the same inputs into one launch."""
        sink = self.__dict__.get("_moments_sink")
        if sink is not None and plan.deferrable():
            sink.append(plan)
        else:
            plan.run()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class MeanSquaredError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0
    sum_squared_error: Tensor
    total: Tensor

    def __init__(self, squared: bool = True, num_outputs: int = 1, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(squared, bool):
            raise ValueError(f"Expected argument `squared` to be a boolean but got {squared}")
        self.squared = squared
        if not (isinstance(num_outputs, int) and num_outputs > 0):
            raise ValueError(f"Expected num_outputs to be a positive integer but got {num_outputs}")
        self.num_outputs = num_outputs
        self.add_state("sum_squared_error", default=torch.zeros(num_outputs), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0), dist_reduce_fx="sum")
        self._moments = [("sum_squared_error", ops.SSE), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        _check_data_shape_to_num_outputs(preds, target, self.num_outputs, allow_1d_reshape=True)
        self._fused_update(preds, target, self.num_outputs)

    def compute(self) -> Tensor:
        sse = self.sum_squared_error.squeeze() if self.num_outputs == 1 else self.sum_squared_error
        return _mean_squared_error_compute(sse, self.total, squared=self.squared)


class MeanAbsoluteError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("sum_abs_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0), dist_reduce_fx="sum")
        self._moments = [("sum_abs_error", ops.SAE), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        self._fused_update(preds, target)

    def compute(self) -> Tensor:
        return _mean_absolute_error_compute(self.sum_abs_error, self.total)


class MeanAbsolutePercentageError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("sum_abs_per_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0.0), dist_reduce_fx="sum")
        self._moments = [("sum_abs_per_error", ops.MAPE), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        self._fused_update(preds, target)

    def compute(self) -> Tensor:
        return _mean_absolute_percentage_error_compute(self.sum_abs_per_error, self.total)


class SymmetricMeanAbsolutePercentageError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: Optional[float] = None

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("sum_abs_per_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0.0), dist_reduce_fx="sum")
        self._moments = [("sum_abs_per_error", ops.SMAPE), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        self._fused_update(preds, target)

    def compute(self) -> Tensor:
        return _symmetric_mean_absolute_percentage_error_compute(self.sum_abs_per_error, self.total)


class WeightedMeanAbsolutePercentageError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("sum_abs_error", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("sum_scale", default=torch.tensor(0.0), dist_reduce_fx="sum")
        self._moments = [("sum_abs_error", ops.SAE), ("sum_scale", ops.SABST)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        self._fused_update(preds, target)

    def compute(self) -> Tensor:
        return _weighted_mean_absolute_percentage_error_compute(self.sum_abs_error, self.sum_scale)


class MeanSquaredLogError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.add_state("sum_squared_log_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0), dist_reduce_fx="sum")
        self._moments = [("sum_squared_log_error", ops.MSLE), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        self._fused_update(preds, target)

    def compute(self) -> Tensor:
        return _mean_squared_log_error_compute(self.sum_squared_log_error, self.total)


class LogCoshError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, num_outputs: int = 1, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(num_outputs, int) and num_outputs < 1:
            raise ValueError(f"Expected argument `num_outputs` to be an int larger than 0, but got {num_outputs}")
        self.num_outputs = num_outputs
        self.add_state("sum_log_cosh_error", default=torch.zeros(num_outputs), dist_reduce_fx="sum")
        self.add_state("total", default=torch.tensor(0), dist_reduce_fx="sum")
        self._moments = [("sum_log_cosh_error", ops.LOGCOSH), ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        _check_data_shape_to_num_outputs(preds, target, self.num_outputs)
        self._fused_update(preds, target, self.num_outputs)

    def compute(self) -> Tensor:
        return _log_cosh_error_compute(self.sum_log_cosh_error, self.total)


class R2Score(_MomentsMetric):
    plot_lower_bound: Optional[float] = 0.0
    is_differentiable = True
    higher_is_better = True
    full_state_update = False
    plot_upper_bound: float = 1.0

    def __init__(self, num_outputs: int = 1, adjusted: int = 0, multioutput: str = "uniform_average",
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.num_outputs = num_outputs
        if adjusted < 0 or not isinstance(adjusted, int):
            raise ValueError("`adjusted` parameter should be an integer larger or equal to 0.")
        self.adjusted = adjusted
        allowed = ("raw_values", "uniform_average", "variance_weighted")
        if multioutput not in allowed:
            raise ValueError(
                f"Invalid input to argument `multioutput`. Choose one of the following: {allowed}"
            )
        self.multioutput = multioutput
        self.add_state("sum_squared_error", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("sum_error", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("residual", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0), dist_reduce_fx="sum")
        # reference naming: sum_squared_error = Σt², sum_error = Σt, residual = Σ(t - p)²
        self._moments = [("sum_squared_error", ops.STT), ("sum_error", ops.ST), ("residual", ops.SSE),
                         ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        if preds.ndim > 2:
            raise ValueError(
                "Expected both prediction and target to be 1D or 2D tensors,"
                f" but received tensors with dimension {preds.shape}"
            )
        k = preds.shape[1] if preds.ndim == 2 else 1
        if k != self.num_outputs:
            raise ValueError(f"Expected `num_outputs` ({self.num_outputs}) to match the input dimension ({k}).")
        self._fused_update(preds, target, k)

    def compute(self) -> Tensor:
        sq = lambda x: x.squeeze(0) if self.num_outputs == 1 else x  # noqa: E731
        return _r2_score_compute(sq(self.sum_squared_error), sq(self.sum_error), sq(self.residual), self.total,
                                 self.adjusted, self.multioutput)


class RelativeSquaredError(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False

    def __init__(self, num_outputs: int = 1, squared: bool = True, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.num_outputs = num_outputs
        self.add_state("sum_squared_error", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("sum_error", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("residual", default=torch.zeros(self.num_outputs), dist_reduce_fx="sum")
        self.add_state("total", default=tensor(0), dist_reduce_fx="sum")
        self.squared = squared
        self._moments = [("sum_squared_error", ops.STT), ("sum_error", ops.ST), ("residual", ops.SSE),
                         ("total", ops.COUNT)]

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        k = preds.shape[1] if preds.ndim == 2 else 1
        self._fused_update(preds, target, k)

    def compute(self) -> Tensor:
        return _relative_squared_error_compute(self.sum_squared_error, self.sum_error, self.residual, self.total,
                                               squared=self.squared)


class ExplainedVariance(_MomentsMetric):
    plot_lower_bound: Optional[float] = 0.0
    is_differentiable = True
    higher_is_better = True
    full_state_update = False
    plot_upper_bound: float = 1.0

    def __init__(self, multioutput: str = "uniform_average", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        allowed = ("raw_values", "uniform_average", "variance_weighted")
        if multioutput not in allowed:
            raise ValueError(f"Invalid input to argument `multioutput`. Choose one of the following: {allowed}")
        self.multioutput = multioutput
        self.add_state("sum_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("sum_squared_error", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("sum_target", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("sum_squared_target", default=tensor(0.0), dist_reduce_fx="sum")
        self.add_state("num_obs", default=tensor(0.0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        _check_same_shape(preds, target)
        k = preds.shape[1] if preds.ndim == 2 else 1
        n = preds.shape[0]
        if self.sum_error.numel() != k:
            # multi-output: states take the per-output shape on the first update (as the reference's broadcasting)
            for name in ("sum_error", "sum_squared_error", "sum_target", "sum_squared_target"):
                setattr(self, name, getattr(self, name) + torch.zeros(k, dtype=getattr(self, name).dtype,
                                                                       device=preds.device))
        dests = [self.sum_error, self.sum_squared_error, self.sum_target, self.sum_squared_target, self.num_obs]
        if preds.is_cuda and ops.states_ready(self.__dict__, tuple(dests), preds.get_device(),
                                              (torch.float32, torch.float64)):
            # Σ(t - p), Σ(p - t)², Σt, Σt², count: all added into the states by the moments finalize launch
            self._submit(ops.MomentsPlan(preds.reshape(n, k), target.reshape(n, k), k, dests, _EV_IDS,
                                         src=(preds, target), checked=True))
            return
        s = ops.moments_update(preds.reshape(n, k), target.reshape(n, k), k, [ops.SP, ops.ST, ops.SSE, ops.STT], [],
                               [], want_sums=True)
        sq = (lambda x: x[0]) if preds.ndim == 1 else (lambda x: x)
        dt = self.sum_error.dtype
        self.sum_error = self.sum_error + sq(s[:, ops.ST] - s[:, ops.SP]).to(dt)
        self.sum_squared_error = self.sum_squared_error + sq(s[:, ops.SSE]).to(dt)
        self.sum_target = self.sum_target + sq(s[:, ops.ST]).to(dt)
        self.sum_squared_target = self.sum_squared_target + sq(s[:, ops.STT]).to(dt)
        self.num_obs = self.num_obs + n

    def compute(self) -> Union[Tensor, Sequence[Tensor]]:
        return _explained_variance_compute(self.num_obs, self.sum_error, self.sum_squared_error, self.sum_target,
                                           self.sum_squared_target, self.multioutput)


class MinkowskiDistance(_MomentsMetric):
    is_differentiable = True
    higher_is_better = False
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, p: float, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not (isinstance(p, (float, int)) and p >= 1):
            raise TorchMetricsUserError(f"Argument ``p`` must be a float or int greater than 1, but got {p}")
        self.p = p
        self._power = float(p)
        self.add_state("minkowski_dist_sum", default=tensor(0.0), dist_reduce_fx="sum")
        self._moments = [("minkowski_dist_sum", ops.MINK)]

    def update(self, preds: Tensor, targets: Tensor) -> None:
        _check_same_shape(preds, targets)
        self._fused_update(preds, targets)

    def compute(self) -> Tensor:
        return _minkowski_distance_compute(self.minkowski_dist_sum, self.p)


class TweedieDevianceScore(Metric):
    is_differentiable = True
    higher_is_better = None
    full_state_update = False
    plot_lower_bound: float = 0.0

    def __init__(self, power: float = 0.0, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if 0 < power < 1:
            raise ValueError(f"Deviance Score is not defined for power={power}.")
        self.power: float = power
        self.add_state("sum_deviance_score", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("num_observations", torch.tensor(0), dist_reduce_fx="sum")

    def update(self, preds: Tensor, targets: Tensor) -> None:
        s, n = _tweedie_deviance_score_update(preds, targets, self.power)
        self.sum_deviance_score += s
        self.num_observations += n

    def compute(self) -> Tensor:
        return _tweedie_deviance_score_compute(self.sum_deviance_score, self.num_observations)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class CriticalSuccessIndex(Metric):
    is_differentiable = False
    higher_is_better = True

    def __init__(self, threshold: float, keep_sequence_dim: Optional[int] = None, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.threshold = float(threshold)
        if keep_sequence_dim and (not isinstance(keep_sequence_dim, int) or keep_sequence_dim < 0):
            raise ValueError(f"Expected keep_sequence_dim to be a non-negative integer but got {keep_sequence_dim}")
        self.keep_sequence_dim = keep_sequence_dim
        if keep_sequence_dim is None:
            self.add_state("hits", default=torch.tensor(0), dist_reduce_fx="sum")
            self.add_state("misses", default=torch.tensor(0), dist_reduce_fx="sum")
            self.add_state("false_alarms", default=torch.tensor(0), dist_reduce_fx="sum")
        else:
            self.add_state("hits_list", default=[], dist_reduce_fx="cat")
            self.add_state("misses_list", default=[], dist_reduce_fx="cat")
            self.add_state("false_alarms_list", default=[], dist_reduce_fx="cat")

    def update(self, preds: Tensor, target: Tensor) -> None:
        hits, misses, fa = _critical_success_index_update(preds, target, self.threshold, self.keep_sequence_dim)
        if self.keep_sequence_dim is None:
            self.hits += hits
            self.misses += misses
            self.false_alarms += fa
        else:
            self.hits_list.append(hits)
            self.misses_list.append(misses)
            self.false_alarms_list.append(fa)

    def compute(self) -> Tensor:
        if self.keep_sequence_dim is None:
            return _critical_success_index_compute(self.hits, self.misses, self.false_alarms)
        return _critical_success_index_compute(
            dim_zero_cat(self.hits_list), dim_zero_cat(self.misses_list), dim_zero_cat(self.false_alarms_list)
        )
