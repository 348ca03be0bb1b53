"""Numerically safe helpers (parity: reference ``S/utilities/compute.py:20-157``).

Note: the reference ``_safe_divide`` mutates ``denom`` in place (``compute.py:52``); ours is side-effect free and
produces identical values.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor


def _safe_matmul(x: Tensor, y: Tensor) -> Tensor:
    """``x @ y.T`` with fp16 inputs promoted to fp32 for the product."""
    if x.dtype == torch.float16 or y.dtype == torch.float16:
        return (x.float() @ y.T.float()).half()
    return x @ y.T


def _safe_xlogy(x: Tensor, y: Tensor) -> Tensor:
    """``x * log(y)`` with the convention ``0 * log(.) = 0``."""
    res = x * torch.log(y)
    return torch.where(x == 0, torch.zeros_like(res), res)


def _safe_divide(num: Tensor, denom: Tensor) -> Tensor:
    """``num / denom`` with zero denominators treated as 1 (so 0/0 -> 0). Integer inputs are promoted to float."""
    num = num if num.is_floating_point() else num.float()
    denom = denom if denom.is_floating_point() else denom.float()
    denom = torch.where(denom == 0, torch.ones_like(denom), denom)
    return num / denom


def _adjust_weights_safe_divide(
    score: Tensor, average: Optional[str], multilabel: bool, tp: Tensor, fp: Tensor, fn: Tensor
) -> Tensor:
    """Macro / weighted averaging of per-class scores; classes with no support are dropped (non-multilabel)."""
    if average is None or average == "none":
        return score
    if average == "weighted":
        weights = tp + fn
    else:
        weights = torch.ones_like(score)
        if not multilabel:
            weights = torch.where(tp + fp + fn == 0, torch.zeros_like(weights), weights)
    return _safe_divide(weights * score, weights.sum(-1, keepdim=True)).sum(-1)


def _auc_format_inputs(x: Tensor, y: Tensor) -> Tuple[Tensor, Tensor]:
    x, y = (t.squeeze() if t.ndim > 1 else t for t in (x, y))
    if max(x.ndim, y.ndim) > 1:
        raise ValueError(
            f"Expected both `x` and `y` tensor to be 1d, but got tensors with dimension {x.ndim} and {y.ndim}"
        )
    if x.numel() != y.numel():
        raise ValueError(
            f"Expected the same number of elements in `x` and `y` tensor but received {x.numel()} and {y.numel()}"
        )
    return x, y


def _auc_compute_without_check(x: Tensor, y: Tensor, direction: float, axis: int = -1) -> Tensor:
    """Trapezoidal area, assuming ``x`` is monotone in the given ``direction``."""
    with torch.no_grad():
        return torch.trapz(y, x, dim=axis) * direction


def _auc_compute(x: Tensor, y: Tensor, reorder: bool = False) -> Tensor:
    with torch.no_grad():
        if reorder:
            x, order = torch.sort(x, stable=True)
            y = y[order]
        direction = 1.0
        if x.numel() > 1:
            # both monotonicity tests in one host read
            dx = x.diff()
            falls, non_increasing = torch.stack([(dx < 0).any(), (dx <= 0).all()]).tolist()
            if falls:
                if not non_increasing:
                    raise ValueError(
                        "The `x` tensor is neither increasing or decreasing. Try setting the reorder argument to `True`."
                    )
                direction = -1.0
        return _auc_compute_without_check(x, y, direction)


def auc(x: Tensor, y: Tensor, reorder: bool = False) -> Tensor:
    """Area under a curve by the trapezoidal rule."""
    x, y = _auc_format_inputs(x, y)
    return _auc_compute(x, y, reorder=reorder)


def interp(x: Tensor, xp: Tensor, fp: Tensor) -> Tensor:
    """Piecewise-linear interpolation of ``(xp, fp)`` at ``x``, extrapolating at the ends.

    The segment of ``x[j]`` is ``#{i : x[j] >= xp[i]} - 1`` clamped to ``[0, len(xp) - 2]``, as in the reference
    (``S/utilities/compute.py:154``: a count over the whole curve, so a non-monotone ``xp`` picks the same segment).  The
    count is taken as a binary search over a sorted copy of ``xp`` (NaN sorts last and counts for nothing) instead of
    the reference's ``[len(x), len(xp)]`` comparison matrix."""
    slope = _safe_divide(fp[1:] - fp[:-1], xp[1:] - xp[:-1])
    icpt = fp[:-1] - slope * xp[:-1]
    xs = xp.contiguous().sort().values
    xc = x.contiguous()
    cnt = torch.searchsorted(xs.nan_to_num(nan=float("inf")), xc, right=True)
    # a NaN xp is never counted (NaN -> +inf above would count it for x = +inf); a NaN x counts nothing
    cnt = torch.minimum(cnt, (~torch.isnan(xs)).sum()).masked_fill(torch.isnan(xc), 0)
    idx = (cnt - 1).clamp(0, slope.numel() - 1)
    return slope[idx] * x + icpt[idx]


__all__ = ["auc", "interp"]
