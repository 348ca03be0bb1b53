"""Pixel / band statistics: PSNR, PSNR-B, SAM, ERGAS, total variation, image gradients, RMSE-SW, RASE.

Behavioural references: ``F/image/psnr.py``, ``psnrb.py``, ``sam.py``, ``ergas.py``, ``tv.py``, ``gradients.py``,
``rmse_sw.py``, ``rase.py``.  On ROCm, RMSE-SW / RASE maps come from one box-window kernel launch over all channels
and images, and PSNR-B's SSE + blocking-effect sums and total variation from one neighbour-difference pass
(``csrc/image/window_stats.hip``); on CPU all channels are filtered by one grouped convolution (the reference loops over
channels in Python) and the blocking-effect factor is built from strided views instead of index lists.
"""
import math
from typing import Optional, Tuple, Union

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_amd import ops
from torchmetrics_amd.functional.image.helper import _uniform_filter
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.distributed import reduce
from torchmetrics_amd.utilities.prints import rank_zero_warn


# ---------------------------------------------------------------------------------------------------------- PSNR
def _psnr_compute(sum_squared_error: Tensor, num_obs: Tensor, data_range: Tensor, base: float = 10.0,
                  reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    psnr_base_e = 2 * torch.log(data_range) - torch.log(sum_squared_error / num_obs)
    return reduce(psnr_base_e * (10 / math.log(base)), reduction=reduction)


def _psnr_update(preds: Tensor, target: Tensor,
                 dim: Optional[Union[int, Tuple[int, ...]]] = None) -> Tuple[Tensor, Tensor]:
    if dim is None:
        return torch.sum((preds - target) ** 2), torch.tensor(target.numel(), device=target.device)
    diff = preds - target
    sse = torch.sum(diff * diff, dim=dim)
    dims = [dim] if isinstance(dim, int) else list(dim)
    if not dims:
        num_obs = torch.tensor(target.numel(), device=target.device)
    else:
        num_obs = torch.tensor(target.size(), device=target.device)[dims].prod().expand_as(sse)
    return sse, num_obs


def peak_signal_noise_ratio(
    preds: Tensor,
    target: Tensor,
    data_range: Optional[Union[float, Tuple[float, float]]] = None,
    base: float = 10.0,
    reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean",
    dim: Optional[Union[int, Tuple[int, ...]]] = None,
) -> Tensor:
    """Peak signal-to-noise ratio in dB (``base`` 10)."""
    if dim is None and reduction != "elementwise_mean":
        rank_zero_warn(f"The `reduction={reduction}` will not have any effect when `dim` is None.")
    if data_range is None:
        if dim is not None:
            raise ValueError("The `data_range` must be given when `dim` is not None.")
        data_range = target.max() - target.min()
    elif isinstance(data_range, tuple):
        preds = torch.clamp(preds, min=data_range[0], max=data_range[1])
        target = torch.clamp(target, min=data_range[0], max=data_range[1])
        data_range = torch.tensor(data_range[1] - data_range[0])
    else:
        data_range = torch.tensor(float(data_range))
    sse, num_obs = _psnr_update(preds, target, dim=dim)
    return _psnr_compute(sse, num_obs, data_range, base=base, reduction=reduction)


# ------------------------------------------------------------------------------------------------------- PSNR-B
def _compute_bef(x: Tensor, block_size: int = 8) -> Tensor:
    """Blocking effect factor of grayscale images: boundary vs non-boundary neighbour differences."""
    _, channels, height, width = x.shape
    if channels > 1:
        raise ValueError(f"`psnrb` metric expects grayscale images, but got images with {channels} channels.")
    dh = (x[..., :, 1:] - x[..., :, :-1]).pow(2)  # horizontal neighbour differences, column j vs j+1
    dv = (x[..., 1:, :] - x[..., :-1, :]).pow(2)
    hb = torch.zeros(width - 1, dtype=torch.bool, device=x.device)
    hb[block_size - 1::block_size] = True
    vb = torch.zeros(height - 1, dtype=torch.bool, device=x.device)
    vb[block_size - 1::block_size] = True
    d_b = dh[..., hb].sum() + dv[..., vb, :].sum()
    d_bc = dh[..., ~hb].sum() + dv[..., ~vb, :].sum()
    return _bef_from_sums(d_b, d_bc, height, width, block_size)


def _psnrb_compute(sum_squared_error: Tensor, bef: Tensor, num_obs: Tensor, data_range: Tensor) -> Tensor:
    mse = sum_squared_error / num_obs + bef
    peak = torch.where(data_range > 2, data_range**2, torch.ones_like(data_range))
    return 10 * torch.log10(peak / mse)


def _bef_from_sums(d_b: Tensor, d_bc: Tensor, height: int, width: int, block_size: int) -> Tensor:
    n_hb = height * (width / block_size) - 1
    n_hbc = (height * (width - 1)) - n_hb
    n_vb = width * (height / block_size) - 1
    n_vbc = (width * (height - 1)) - n_vb
    d_b = d_b / (n_hb + n_vb)
    d_bc = d_bc / (n_hbc + n_vbc)
    t = math.log2(block_size) / math.log2(min(height, width))
    return torch.where(d_b > d_bc, t * (d_b - d_bc), torch.zeros_like(d_b))


def _psnrb_update(preds: Tensor, target: Tensor, block_size: int = 8) -> Tuple[Tensor, Tensor, Tensor]:
    stats = ops.neighbour_diff_stats(preds, target, block_size, True) if preds.shape[1] == 1 else None
    if stats is not None:
        # ROCm: SSE and the four blocking-effect sums in one pass (csrc/image/window_stats.hip)
        s = stats.sum(0)
        bef = _bef_from_sums(s[1] + s[3], s[2] + s[4], preds.shape[2], preds.shape[3], block_size)
        return s[0].to(preds.dtype), bef.to(preds.dtype), torch.tensor(target.numel(), device=target.device)
    sse = torch.sum((preds - target) ** 2)
    return sse, _compute_bef(preds, block_size=block_size), torch.tensor(target.numel(), device=target.device)


def peak_signal_noise_ratio_with_blocked_effect(preds: Tensor, target: Tensor, block_size: int = 8) -> Tensor:
    """PSNR corrected for JPEG-style blocking artefacts (grayscale)."""
    data_range = target.max() - target.min()
    sse, bef, num_obs = _psnrb_update(preds, target, block_size=block_size)
    return _psnrb_compute(sse, bef, num_obs, data_range)


# ------------------------------------------------------------------------------------------------ SAM / ERGAS
def _same_dtype_4d(preds: Tensor, target: Tensor) -> None:
    if preds.dtype != target.dtype:
        raise TypeError(
            "Expected `preds` and `target` to have the same data type."
            f" Got preds: {preds.dtype} and target: {target.dtype}."
        )
    _check_same_shape(preds, target)
    if len(preds.shape) != 4:
        raise ValueError(
            "Expected `preds` and `target` to have BxCxHxW shape."
            f" Got preds: {preds.shape} and target: {target.shape}."
        )


def _sam_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _same_dtype_4d(preds, target)
    if (preds.shape[1] <= 1) or (target.shape[1] <= 1):
        raise ValueError(
            "Expected channel dimension of `preds` and `target` to be larger than 1."
            f" Got preds: {preds.shape[1]} and target: {target.shape[1]}."
        )
    return preds, target


def _sam_compute(preds: Tensor, target: Tensor,
                 reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    """ROCm (no autograd graph needed): one pass over the channels per pixel (``ops.sam_angles``); else the
    reference's formulation (``F/image/sam.py:56-83``)."""
    if reduction not in ("elementwise_mean", "sum", "none", None):
        raise ValueError("Reduction parameter unknown.")
    fused = ops.sam_angles(preds, target, want_map=reduction in ("none", None),
                           want_sum=reduction in ("elementwise_mean", "sum"))
    if fused is not None:
        amap, total = fused
        if amap is not None:
            return amap
        n = preds.shape[0] * preds.shape[2] * preds.shape[3]
        return (total / n if reduction == "elementwise_mean" else total).to(preds.dtype)
    cos = (preds * target).sum(dim=1) / (preds.norm(dim=1) * target.norm(dim=1))
    return reduce(torch.clamp(cos, -1, 1).acos(), reduction)


def spectral_angle_mapper(preds: Tensor, target: Tensor,
                          reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    """Per-pixel angle between spectral vectors (radians)."""
    preds, target = _sam_update(preds, target)
    return _sam_compute(preds, target, reduction)


def _ergas_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    _same_dtype_4d(preds, target)
    return preds, target


def _ergas_compute(preds: Tensor, target: Tensor, ratio: float = 4,
                   reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean") -> Tensor:
    b, c, h, w = preds.shape
    st = ops.band_stats(preds, target)  # ROCm: per (image, band) Σ(p - t)² and Σt in one pass, fp64
    if st is not None:
        hw = h * w
        rmse_band = torch.sqrt(st[..., 0] / hw)
        score = (100 * ratio * torch.sqrt(torch.sum((rmse_band / (st[..., 1] / hw)) ** 2, dim=1) / c)).to(preds.dtype)
        return reduce(score, reduction)
    p, t = preds.reshape(b, c, h * w), target.reshape(b, c, h * w)
    rmse_band = torch.sqrt(((p - t) ** 2).sum(dim=2) / (h * w))
    score = 100 * ratio * torch.sqrt(torch.sum((rmse_band / t.mean(dim=2)) ** 2, dim=1) / c)
    return reduce(score, reduction)


def error_relative_global_dimensionless_synthesis(
    preds: Tensor, target: Tensor, ratio: float = 4,
    reduction: Literal["elementwise_mean", "sum", "none", None] = "elementwise_mean",
) -> Tensor:
    """ERGAS: relative dimensionless global error of a pansharpened / synthesised image."""
    preds, target = _ergas_update(preds, target)
    return _ergas_compute(preds, target, ratio, reduction)


# ------------------------------------------------------------------------------------------------- TV / grads
def _total_variation_update(img: Tensor) -> Tuple[Tensor, int]:
    if img.ndim != 4:
        raise RuntimeError(f"Expected input `img` to be an 4D tensor, but got {img.shape}")
    stats = ops.neighbour_diff_stats(img, None, 1, False) if img.is_floating_point() else None
    if stats is not None:  # ROCm: both shifted-difference sums in one pass
        return stats[:, 1:].sum(1).to(img.dtype), img.shape[0]
    score = (img[..., 1:, :] - img[..., :-1, :]).abs().sum([1, 2, 3]) + \
        (img[..., :, 1:] - img[..., :, :-1]).abs().sum([1, 2, 3])
    return score, img.shape[0]


def _total_variation_compute(score: Tensor, num_elements: Union[int, Tensor],
                             reduction: Optional[Literal["mean", "sum", "none"]]) -> Tensor:
    if reduction == "mean":
        return score.sum() / num_elements
    if reduction == "sum":
        return score.sum()
    if reduction is None or reduction == "none":
        return score
    raise ValueError("Expected argument `reduction` to either be 'sum', 'mean', 'none' or None")


def total_variation(img: Tensor, reduction: Optional[Literal["mean", "sum", "none"]] = "sum") -> Tensor:
    """Anisotropic total variation (sum of absolute neighbour differences)."""
    score, n = _total_variation_update(img)
    return _total_variation_compute(score, n, reduction)


def _image_gradients_validate(img: Tensor) -> None:
    if not isinstance(img, Tensor):
        raise TypeError(f"The `img` expects a value of <Tensor> type but got {type(img)}")
    if img.ndim != 4:
        raise RuntimeError(f"The `img` expects a 4D tensor but got {img.ndim}D tensor")


def _compute_image_gradients(img: Tensor) -> Tuple[Tensor, Tensor]:
    dy = torch.zeros_like(img)
    dx = torch.zeros_like(img)
    dy[..., :-1, :] = img[..., 1:, :] - img[..., :-1, :]
    dx[..., :, :-1] = img[..., :, 1:] - img[..., :, :-1]
    return dy, dx


def image_gradients(img: Tensor) -> Tuple[Tensor, Tensor]:
    """Forward differences ``(dy, dx)`` with a zero last row / column."""
    _image_gradients_validate(img)
    return _compute_image_gradients(img)


# ----------------------------------------------------------------------------------------------- RMSE-SW / RASE
def _rmse_sw_update(
    preds: Tensor,
    target: Tensor,
    window_size: int,
    rmse_val_sum: Optional[Tensor],
    rmse_map: Optional[Tensor],
    total_images: Optional[Tensor],
) -> Tuple[Tensor, Tensor, Tensor]:
    if preds.dtype != target.dtype:
        raise TypeError(
            f"Expected `preds` and `target` to have the same data type. But got {preds.dtype} and {target.dtype}."
        )
    _check_same_shape(preds, target)
    if len(preds.shape) != 4:
        raise ValueError(f"Expected `preds` and `target` to have BxCxHxW shape. But got {preds.shape}.")
    crop = round(window_size / 2)
    if crop >= target.shape[2] or crop >= target.shape[3]:
        raise ValueError(
            f"Parameter `round(window_size / 2)` is expected to be smaller than {min(target.shape[2], target.shape[3])}"
            f" but got {crop}."
        )
    total_images = (total_images + target.shape[0]) if total_images is not None else torch.tensor(
        target.shape[0], device=target.device)
    maps = ops.box_rmse_maps(preds, target, window_size, False)
    if maps is not None:  # ROCm: the batch-summed map straight from the box-window kernel
        local_sum = maps[0]
    else:
        local_sum = torch.sqrt(_uniform_filter((target - preds) ** 2, window_size)).sum(0)
    val = local_sum[:, crop:-crop, crop:-crop].mean()
    rmse_val_sum = val if rmse_val_sum is None else rmse_val_sum + val
    rmse_map = local_sum if rmse_map is None else rmse_map + local_sum
    return rmse_val_sum, rmse_map, total_images


def _rmse_sw_compute(rmse_val_sum: Optional[Tensor], rmse_map: Tensor,
                     total_images: Tensor) -> Tuple[Optional[Tensor], Tensor]:
    rmse = rmse_val_sum / total_images if rmse_val_sum is not None else None
    if rmse_map is not None:
        rmse_map = rmse_map / total_images
    return rmse, rmse_map


def root_mean_squared_error_using_sliding_window(
    preds: Tensor, target: Tensor, window_size: int = 8, return_rmse_map: bool = False
) -> Union[Optional[Tensor], Tuple[Optional[Tensor], Tensor]]:
    """RMSE over sliding windows (mean over the crop-free interior)."""
    if not isinstance(window_size, int) or window_size < 1:
        raise ValueError("Argument `window_size` is expected to be a positive integer.")
    val, rmse_map, total = _rmse_sw_update(preds, target, window_size, None, None, None)
    rmse, rmse_map = _rmse_sw_compute(val, rmse_map, total)
    return (rmse, rmse_map) if return_rmse_map else rmse


def _rase_update(preds: Tensor, target: Tensor, window_size: int, rmse_map: Tensor, target_sum: Tensor,
                 total_images: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    maps = ops.box_rmse_maps(preds, target, window_size, True) if preds.shape == target.shape and \
        preds.ndim == 4 and preds.dtype == target.dtype else None
    if maps is not None and round(window_size / 2) < min(target.shape[2], target.shape[3]):
        # ROCm: both filtered maps from ONE pass of the box-window kernel
        total_images = total_images + target.shape[0]
        return rmse_map + maps[0], target_sum + maps[1], total_images
    _, rmse_map, total_images = _rmse_sw_update(preds, target, window_size, None, rmse_map, total_images)
    target_sum = target_sum + torch.sum(_uniform_filter(target, window_size) / (window_size**2), dim=0)
    return rmse_map, target_sum, total_images


def _rase_compute(rmse_map: Tensor, target_sum: Tensor, total_images: Tensor, window_size: int) -> Tensor:
    _, rmse_map = _rmse_sw_compute(None, rmse_map, total_images)
    target_mean = (target_sum / total_images).mean(0)
    rase_map = 100 / target_mean * torch.sqrt(torch.mean(rmse_map**2, 0))
    crop = round(window_size / 2)
    return torch.mean(rase_map[crop:-crop, crop:-crop])


def relative_average_spectral_error(preds: Tensor, target: Tensor, window_size: int = 8) -> Tensor:
    """RASE: relative average spectral error over sliding windows."""
    if not isinstance(window_size, int) or window_size < 1:
        raise ValueError("Argument `window_size` is expected to be a positive integer.")
    shape = target.shape[1:]
    rmse_map = torch.zeros(shape, dtype=target.dtype, device=target.device)
    target_sum = torch.zeros(shape, dtype=target.dtype, device=target.device)
    total = torch.tensor(0.0, device=target.device)
    rmse_map, target_sum, total = _rase_update(preds, target, window_size, rmse_map, target_sum, total)
    return _rase_compute(rmse_map, target_sum, total, window_size)
