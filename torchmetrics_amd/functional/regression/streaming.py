"""Streaming (sum-state) regression metrics, functional API.

Parity: reference ``F/regression/{mse,mae,mape,symmetric_mape,wmape,log_mse,log_cosh,r2,rse,explained_variance,
minkowski,tweedie_deviance,csi}.py``.  Every ``_*_update`` is a single pass of the fused moments kernel
(``csrc/regression/moments.hip``) returning fp64-accumulated sums; the ``_*_compute`` functions hold the closed forms.
"""
from typing import Optional, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.compute import _safe_divide, _safe_xlogy
from torchmetrics_amd.utilities.exceptions import TorchMetricsUserError
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils.deferred import raise_if

EPS = 1.17e-06


def _check_data_shape_to_num_outputs(
    preds: Tensor, target: Tensor, num_outputs: int, allow_1d_reshape: bool = False
) -> None:
    if preds.ndim > 2 or target.ndim > 2:
        raise ValueError(
            f"Expected both predictions and target to be either 1- or 2-dimensional tensors,"
            f" but got {target.ndim} and {preds.ndim}."
        )
    bad1 = not allow_1d_reshape and num_outputs == 1 and not (preds.ndim == 1 or preds.shape[1] == 1)
    bad2 = num_outputs > 1 and preds.ndim > 1 and num_outputs != preds.shape[1]
    if bad1 or bad2:
        raise ValueError(
            f"Expected argument `num_outputs` to match the second dimension of input, but got {num_outputs}"
            f" and {preds.shape[1]}."
        )


def _sums(preds: Tensor, target: Tensor, k: int, ids: list, eps: float = EPS, power: float = 2.0,
          shift_p: Optional[Tensor] = None, shift_t: Optional[Tensor] = None) -> Tensor:
    """``[k, 14]`` fp64 sums of the given ids for ``[N, k]`` inputs (one fused kernel pass on ROCm)."""
    return ops.moments_update(preds, target, k, ids, [], [], eps=eps, power=power, shift_p=shift_p, shift_t=shift_t,
                              want_sums=True)


def _out_dtype(preds: Tensor, target: Tensor) -> torch.dtype:
    dt = torch.promote_types(preds.dtype, target.dtype)
    return dt if dt.is_floating_point else torch.get_default_dtype()


# ------------------------------------------------------------------------------------------------------------ MSE
def _mean_squared_error_update(preds: Tensor, target: Tensor, num_outputs: int) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs, allow_1d_reshape=True)
    k = num_outputs if num_outputs > 1 else 1
    s = _sums(preds.reshape(-1, k), target.reshape(-1, k), k, [ops.SSE])
    sse = s[:, ops.SSE].to(_out_dtype(preds, target))
    n = target.numel() if num_outputs == 1 else target.shape[0]
    return (sse[0] if num_outputs == 1 else sse), n


def _mean_squared_error_compute(sum_squared_error: Tensor, total: Union[int, Tensor], squared: bool = True) -> Tensor:
    return ops.ratio(sum_squared_error, total, take_sqrt=not squared)


def mean_squared_error(preds: Tensor, target: Tensor, squared: bool = True, num_outputs: int = 1) -> Tensor:
    sse, n = _mean_squared_error_update(preds, target, num_outputs)
    return _mean_squared_error_compute(sse, n, squared)


# ------------------------------------------------------------------------------------------------------------ MAE
def _mean_absolute_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    s = _sums(preds.reshape(-1), target.reshape(-1), 1, [ops.SAE])
    return s[0, ops.SAE].to(_out_dtype(preds, target)), target.numel()


def _mean_absolute_error_compute(sum_abs_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return ops.ratio(sum_abs_error, num_obs)


def mean_absolute_error(preds: Tensor, target: Tensor) -> Tensor:
    return _mean_absolute_error_compute(*_mean_absolute_error_update(preds, target))


# ------------------------------------------------------------------------------------------------ MAPE / SMAPE / WMAPE
def _mean_absolute_percentage_error_update(preds: Tensor, target: Tensor, epsilon: float = EPS) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    s = _sums(preds.reshape(-1), target.reshape(-1), 1, [ops.MAPE], eps=epsilon)
    return s[0, ops.MAPE].to(_out_dtype(preds, target)), target.numel()


def _mean_absolute_percentage_error_compute(sum_abs_per_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_abs_per_error / num_obs


def mean_absolute_percentage_error(preds: Tensor, target: Tensor) -> Tensor:
    return _mean_absolute_percentage_error_compute(*_mean_absolute_percentage_error_update(preds, target))


def _symmetric_mean_absolute_percentage_error_update(
    preds: Tensor, target: Tensor, epsilon: float = EPS
) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    s = _sums(preds.reshape(-1), target.reshape(-1), 1, [ops.SMAPE], eps=epsilon)
    return s[0, ops.SMAPE].to(_out_dtype(preds, target)), target.numel()


def _symmetric_mean_absolute_percentage_error_compute(sum_abs_per_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_abs_per_error / num_obs


def symmetric_mean_absolute_percentage_error(preds: Tensor, target: Tensor) -> Tensor:
    return _symmetric_mean_absolute_percentage_error_compute(
        *_symmetric_mean_absolute_percentage_error_update(preds, target)
    )


def _weighted_mean_absolute_percentage_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    s = _sums(preds.reshape(-1), target.reshape(-1), 1, [ops.SAE, ops.SABST])
    dt = _out_dtype(preds, target)
    return s[0, ops.SAE].to(dt), s[0, ops.SABST].to(dt)


def _weighted_mean_absolute_percentage_error_compute(
    sum_abs_error: Tensor, sum_scale: Tensor, epsilon: float = EPS
) -> Tensor:
    return sum_abs_error / torch.clamp(sum_scale, min=epsilon)


def weighted_mean_absolute_percentage_error(preds: Tensor, target: Tensor) -> Tensor:
    return _weighted_mean_absolute_percentage_error_compute(
        *_weighted_mean_absolute_percentage_error_update(preds, target)
    )


# ------------------------------------------------------------------------------------------------------ MSLE / logcosh
def _mean_squared_log_error_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, int]:
    _check_same_shape(preds, target)
    s = _sums(preds.reshape(-1), target.reshape(-1), 1, [ops.MSLE])
    return s[0, ops.MSLE].to(_out_dtype(preds, target)), target.numel()


def _mean_squared_log_error_compute(sum_squared_log_error: Tensor, num_obs: Union[int, Tensor]) -> Tensor:
    return sum_squared_log_error / num_obs


def mean_squared_log_error(preds: Tensor, target: Tensor) -> Tensor:
    return _mean_squared_log_error_compute(*_mean_squared_log_error_update(preds, target))


def _log_cosh_error_update(preds: Tensor, target: Tensor, num_outputs: int) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, target)
    _check_data_shape_to_num_outputs(preds, target, num_outputs)
    k = preds.shape[1] if preds.ndim == 2 else 1
    s = _sums(preds.reshape(-1, k), target.reshape(-1, k), k, [ops.LOGCOSH])
    return s[:, ops.LOGCOSH].to(_out_dtype(preds, target)).squeeze(), torch.tensor(target.shape[0], device=preds.device)


def _log_cosh_error_compute(sum_log_cosh_error: Tensor, num_obs: Tensor) -> Tensor:
    return (sum_log_cosh_error / num_obs).squeeze()


def log_cosh_error(preds: Tensor, target: Tensor) -> Tensor:
    k = preds.shape[1] if preds.ndim == 2 else 1
    return _log_cosh_error_compute(*_log_cosh_error_update(preds, target, k))


# ------------------------------------------------------------------------------------------------------- R2 / RSE
def _r2_score_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor, Tensor, int]:
    _check_same_shape(preds, target)
    if preds.ndim > 2:
        raise ValueError(
            "Expected both prediction and target to be 1D or 2D tensors,"
            f" but received tensors with dimension {preds.shape}"
        )
    k = preds.shape[1] if preds.ndim == 2 else 1
    s = _sums(preds.reshape(-1, k), target.reshape(-1, k), k, [ops.STT, ops.ST, ops.SSE])
    dt = _out_dtype(preds, target)
    sq = lambda x: x if preds.ndim == 2 else x[0]  # noqa: E731
    return sq(s[:, ops.STT].to(dt)), sq(s[:, ops.ST].to(dt)), sq(s[:, ops.SSE].to(dt)), target.size(0)


def _r2_score_compute(
    sum_squared_obs: Tensor,
    sum_obs: Tensor,
    rss: Tensor,
    num_obs: Union[int, Tensor],
    adjusted: int = 0,
    multioutput: str = "uniform_average",
) -> Tensor:
    mo = ops.MULTIOUT_IDS.get(multioutput)
    if mo is not None and sum_obs.is_cuda and ops.regression_computable((sum_squared_obs, sum_obs, rss), num_obs):
        # one launch for the per-output scores and their average (csrc/regression/regression_compute.hip)
        out = ops.regression_compute(ops.REG_R2, (sum_squared_obs, sum_obs, rss), num_obs, mo)
        k = sum_obs.numel()
        # the kernel's flag slot holds n < 2 (a task output: a fused collection compute folds it into its status read)
        raise_if(out[k + 1 : k + 2], ValueError, "Needs at least two samples to calculate r2 score.")
        r2 = out[:k].view(sum_obs.shape) if mo == 0 else out[k]
        return _r2_adjust(r2, num_obs, adjusted)
    if num_obs < 2:
        raise ValueError("Needs at least two samples to calculate r2 score.")
    mean_obs = sum_obs / num_obs
    tss = sum_squared_obs - sum_obs * mean_obs
    nz_rss = ~torch.isclose(rss, torch.zeros_like(rss), atol=1e-4)
    nz_tss = ~torch.isclose(tss, torch.zeros_like(tss), atol=1e-4)
    raw = torch.where(nz_rss & nz_tss, 1 - rss / torch.where(nz_tss, tss, torch.ones_like(tss)), torch.ones_like(rss))
    raw = torch.where(nz_rss & ~nz_tss, torch.zeros_like(raw), raw)
    if multioutput == "raw_values":
        r2 = raw
    elif multioutput == "uniform_average":
        r2 = torch.mean(raw)
    elif multioutput == "variance_weighted":
        r2 = torch.sum(tss / torch.sum(tss) * raw)
    else:
        raise ValueError(
            "Argument `multioutput` must be either `raw_values`,"
            f" `uniform_average` or `variance_weighted`. Received {multioutput}."
        )
    return _r2_adjust(r2, num_obs, adjusted)


def _r2_adjust(r2: Tensor, num_obs: Union[int, Tensor], adjusted: int) -> Tensor:
    if adjusted < 0 or not isinstance(adjusted, int):
        raise ValueError("`adjusted` parameter should be an integer larger or equal to 0.")
    if adjusted != 0:
        if adjusted > num_obs - 1:
            rank_zero_warn(
                "More independent regressions than data points in adjusted r2 score. Falls back to standard r2 score.",
                UserWarning,
            )
        elif adjusted == num_obs - 1:
            rank_zero_warn("Division by zero in adjusted r2 score. Falls back to standard r2 score.", UserWarning)
        else:
            return 1 - (1 - r2) * (num_obs - 1) / (num_obs - adjusted - 1)
    return r2


def r2_score(preds: Tensor, target: Tensor, adjusted: int = 0, multioutput: str = "uniform_average") -> Tensor:
    sum_squared_obs, sum_obs, rss, num_obs = _r2_score_update(preds, target)
    return _r2_score_compute(sum_squared_obs, sum_obs, rss, num_obs, adjusted, multioutput)


def _relative_squared_error_compute(
    sum_squared_obs: Tensor, sum_obs: Tensor, sum_squared_error: Tensor, num_obs: Union[int, Tensor],
    squared: bool = True,
) -> Tensor:
    eps = torch.finfo(sum_squared_error.dtype).eps
    rse = sum_squared_error / torch.clamp(sum_squared_obs - sum_obs * sum_obs / num_obs, min=eps)
    if not squared:
        rse = torch.sqrt(rse)
    return torch.mean(rse)


def relative_squared_error(preds: Tensor, target: Tensor, squared: bool = True) -> Tensor:
    sum_squared_obs, sum_obs, rss, num_obs = _r2_score_update(preds, target)
    return _relative_squared_error_compute(sum_squared_obs, sum_obs, rss, num_obs, squared=squared)


# ---------------------------------------------------------------------------------------------- explained variance
def _explained_variance_update(preds: Tensor, target: Tensor) -> Tuple[int, Tensor, Tensor, Tensor, Tensor]:
    _check_same_shape(preds, target)
    k = preds.shape[1] if preds.ndim == 2 else 1
    # sum_error = Σ(t - p) = Σt - Σp ; the rest directly
    s = _sums(preds.reshape(-1, k), target.reshape(-1, k), k, [ops.SP, ops.ST, ops.SSE, ops.STT])
    dt = _out_dtype(preds, target)
    sq = lambda x: x if preds.ndim == 2 else x[0]  # noqa: E731
    sum_error = (s[:, ops.ST] - s[:, ops.SP]).to(dt)
    return preds.size(0), sq(sum_error), sq(s[:, ops.SSE].to(dt)), sq(s[:, ops.ST].to(dt)), sq(s[:, ops.STT].to(dt))


def _explained_variance_compute(
    num_obs: Union[int, Tensor],
    sum_error: Tensor,
    sum_squared_error: Tensor,
    sum_target: Tensor,
    sum_squared_target: Tensor,
    multioutput: str = "uniform_average",
) -> Tensor:
    states = (sum_error, sum_squared_error, sum_target, sum_squared_target)
    mo = ops.MULTIOUT_IDS.get(multioutput)
    if mo is not None and sum_error.is_cuda and ops.regression_computable(states, num_obs):
        out = ops.regression_compute(ops.REG_EV, states, num_obs, mo)
        k = sum_error.numel()
        return out[:k].view(sum_error.shape) if mo == 0 else out[k]
    diff_avg = sum_error / num_obs
    numerator = sum_squared_error / num_obs - diff_avg * diff_avg
    target_avg = sum_target / num_obs
    denominator = sum_squared_target / num_obs - target_avg * target_avg
    nz_num = numerator != 0
    nz_den = denominator != 0
    scores = torch.where(
        nz_num & nz_den, 1.0 - numerator / torch.where(nz_den, denominator, torch.ones_like(denominator)),
        torch.ones_like(diff_avg),
    )
    scores = torch.where(nz_num & ~nz_den, torch.zeros_like(scores), scores)
    if multioutput == "raw_values":
        return scores
    if multioutput == "uniform_average":
        return torch.mean(scores)
    return torch.sum(denominator / torch.sum(denominator) * scores)


def explained_variance(preds: Tensor, target: Tensor, multioutput: str = "uniform_average") -> Tensor:
    allowed = ("raw_values", "uniform_average", "variance_weighted")
    if multioutput not in allowed:
        raise ValueError(f"Invalid input to argument `multioutput`. Choose one of the following: {allowed}")
    return _explained_variance_compute(*_explained_variance_update(preds, target), multioutput)


# ---------------------------------------------------------------------------------------------- minkowski / tweedie
def _minkowski_distance_update(preds: Tensor, targets: Tensor, p: float) -> Tensor:
    _check_same_shape(preds, targets)
    if not (isinstance(p, (float, int)) and p >= 1):
        raise TorchMetricsUserError(f"Argument ``p`` must be a float or int greater than 1, but got {p}")
    s = _sums(preds.reshape(-1), targets.reshape(-1), 1, [ops.MINK], power=float(p))
    return s[0, ops.MINK].to(_out_dtype(preds, targets))


def _minkowski_distance_compute(distance: Tensor, p: float) -> Tensor:
    return torch.pow(distance, 1.0 / p)


def minkowski_distance(preds: Tensor, targets: Tensor, p: float) -> Tensor:
    return _minkowski_distance_compute(_minkowski_distance_update(preds, targets, p), p)


def _tweedie_deviance_score_update(preds: Tensor, targets: Tensor, power: float = 0.0) -> Tuple[Tensor, Tensor]:
    _check_same_shape(preds, targets)
    if 0 < power < 1:
        raise ValueError(f"Deviance Score is not defined for power={power}.")
    if power == 0:
        dev = torch.pow(targets - preds, exponent=2)
    elif power == 1:
        if torch.any(preds <= 0) or torch.any(targets < 0):
            raise ValueError(f"For power={power}, 'preds' has to be strictly positive and 'targets' cannot be negative.")
        dev = 2 * (_safe_xlogy(targets, targets / preds) + preds - targets)
    elif power == 2:
        if torch.any(preds <= 0) or torch.any(targets <= 0):
            raise ValueError(f"For power={power}, both 'preds' and 'targets' have to be strictly positive.")
        dev = 2 * (torch.log(preds / targets) + (targets / preds) - 1)
    else:
        if power < 0:
            if torch.any(preds <= 0):
                raise ValueError(f"For power={power}, 'preds' has to be strictly positive.")
        elif 1 < power < 2:
            if torch.any(preds <= 0) or torch.any(targets < 0):
                raise ValueError(
                    f"For power={power}, 'targets' has to be strictly positive and 'preds' cannot be negative."
                )
        elif torch.any(preds <= 0) or torch.any(targets <= 0):
            raise ValueError(f"For power={power}, both 'preds' and 'targets' have to be strictly positive.")
        t1 = torch.pow(torch.clamp(targets, min=0), 2 - power) / ((1 - power) * (2 - power))
        t2 = targets * torch.pow(preds, 1 - power) / (1 - power)
        t3 = torch.pow(preds, 2 - power) / (2 - power)
        dev = 2 * (t1 - t2 + t3)
    return torch.sum(dev), torch.tensor(torch.numel(dev), device=preds.device)


def _tweedie_deviance_score_compute(sum_deviance_score: Tensor, num_observations: Tensor) -> Tensor:
    return sum_deviance_score / num_observations


def tweedie_deviance_score(preds: Tensor, targets: Tensor, power: float = 0.0) -> Tensor:
    return _tweedie_deviance_score_compute(*_tweedie_deviance_score_update(preds, targets, power))


# ------------------------------------------------------------------------------------------------------------ CSI
def _critical_success_index_update(
    preds: Tensor, target: Tensor, threshold: float, keep_sequence_dim: Optional[int] = None
) -> Tuple[Tensor, Tensor, Tensor]:
    _check_same_shape(preds, target)
    if keep_sequence_dim is None:
        dims = None
    elif not 0 <= keep_sequence_dim < preds.ndim:
        raise ValueError(f"Expected keep_sequence dim to be in range [0, {preds.ndim}] but got {keep_sequence_dim}")
    else:
        dims = tuple(i for i in range(preds.ndim) if i != keep_sequence_dim)
    pb = preds >= threshold
    tb = target >= threshold
    hits = pb & tb
    misses = ~pb & tb
    false_alarms = pb & ~tb
    if dims is None:
        return hits.sum().int(), misses.sum().int(), false_alarms.sum().int()
    return hits.sum(dim=dims).int(), misses.sum(dim=dims).int(), false_alarms.sum(dim=dims).int()


def _critical_success_index_compute(hits: Tensor, misses: Tensor, false_alarms: Tensor) -> Tensor:
    return _safe_divide(hits, hits + misses + false_alarms)


def critical_success_index(
    preds: Tensor, target: Tensor, threshold: float, keep_sequence_dim: Optional[int] = None
) -> Tensor:
    return _critical_success_index_compute(*_critical_success_index_update(preds, target, threshold, keep_sequence_dim))
