"""Spatial / pansharpening quality: SCC, VIF, D_lambda, D_s, QNR.

Behavioural references: ``F/image/scc.py``, ``vif.py``, ``d_lambda.py``, ``d_s.py``, ``qnr.py``.  Channel loops of
the reference become grouped convolutions / batched planes; the band-pair UQI matrix of D_lambda is one batched call
of the fused UQI kernel over all ``C(C-1)/2`` pairs; the ``pan`` degradation of D_s is an in-house box filter +
bilinear resize (no torchvision dependency).
"""
import math
from typing import Literal, Optional, Tuple, Union

import torch
import torch.nn.functional as F  # noqa: N812
from torch import Tensor

from torchmetrics_amd import ops

from torchmetrics_amd.functional.image.helper import _symmetric_pad, _uniform_filter
from torchmetrics_amd.functional.image.ssim import _uqi_plane_means
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.distributed import reduce


# ------------------------------------------------------------------------------------------------------------ SCC
def _scc_update(preds: Tensor, target: Tensor, hp_filter: Tensor, window_size: int) -> Tuple[Tensor, Tensor, Tensor]:
    if preds.dtype != target.dtype:
        target = target.to(preds.dtype)
    _check_same_shape(preds, target)
    if preds.ndim not in (3, 4):
        raise ValueError(
            "Expected `preds` and `target` to have batch of colored images with BxCxHxW shape"
            "  or batch of grayscale images of BxHxW shape."
            f" Got preds: {preds.shape} and target: {target.shape}."
        )
    if preds.ndim == 3:
        preds, target = preds.unsqueeze(1), target.unsqueeze(1)
    if not window_size > 0:
        raise ValueError(f"Expected `window_size` to be a positive integer. Got {window_size}.")
    if window_size > preds.size(2) or window_size > preds.size(3):
        raise ValueError(
            f"Expected `window_size` to be less than or equal to the size of the image."
            f" Got window_size: {window_size} and image size: {preds.size(2)}x{preds.size(3)}."
        )
    preds, target = preds.to(torch.float32), target.to(torch.float32)
    return preds, target, hp_filter[None, None, :].to(dtype=preds.dtype, device=preds.device)


def _scc_plane_means(preds: Tensor, target: Tensor, hp_filter: Tensor, window_size: int) -> Tensor:
    """Per-image SCC averaged over channels and pixels, ``[B]``.

    ROCm: after the (symmetric-padded) high-pass convolution, the zero-padded windowed moments and the per-window
    correlation run in one launch of the SSIM window kernel (SCC mode, uniform separable window, per-tile sums); the
    reference stacks 5 maps, runs a grouped conv and forms the map elementwise (``F/image/scc.py:41-90``)."""
    b, c, h, w = preds.shape
    if not (preds.is_cuda and window_size <= 33):
        return _scc_map(preds, target, hp_filter, window_size).mean(dim=[1, 2, 3])
    x = torch.cat([preds, target], 0).reshape(2 * b * c, 1, h, w)
    kh, kw = hp_filter.shape[-2:]
    x = _symmetric_pad(x, 3, (kw - 1) // 2, math.ceil((kw - 1) / 2))
    x = _symmetric_pad(x, 2, (kh - 1) // 2, math.ceil((kh - 1) / 2))
    hp = F.conv2d(x, hp_filter.flip([2, 3])) * 2.0
    lo, hi = math.ceil((window_size - 1) / 2), (window_size - 1) // 2
    hp = F.pad(hp, (lo, hi, lo, hi))[:, 0]
    win = torch.full((window_size,), 1.0 / window_size, dtype=hp.dtype, device=hp.device)
    consts = torch.zeros(3, dtype=hp.dtype, device=hp.device)
    part = ops.ssim2d_partials(hp[: b * c].contiguous(), hp[b * c:].contiguous(), win, win, consts, ops.SCC_MODE)
    per_plane = part.sum(1)[:, 0].to(preds.dtype)
    return per_plane.reshape(b, c).sum(1) / (c * h * w)


def _scc_map(preds: Tensor, target: Tensor, hp_filter: Tensor, window_size: int) -> Tensor:
    """Per-pixel spatial correlation of Laplacian-filtered images, all channels at once: ``[B, C, H, W]``."""
    b, c, h, w = preds.shape
    x = torch.cat([preds, target], 0).reshape(2 * b * c, 1, h, w)
    kh, kw = hp_filter.shape[-2:]
    x = _symmetric_pad(x, 3, (kw - 1) // 2, math.ceil((kw - 1) / 2))
    x = _symmetric_pad(x, 2, (kh - 1) // 2, math.ceil((kh - 1) / 2))
    hp = F.conv2d(x, hp_filter.flip([2, 3])) * 2.0  # true convolution (scipy.signal.convolve2d semantics)
    p_hp, t_hp = hp[: b * c], hp[b * c:]
    lo, hi = math.ceil((window_size - 1) / 2), (window_size - 1) // 2
    win = torch.full((1, 1, window_size, window_size), 1.0 / window_size**2, dtype=hp.dtype, device=hp.device)
    stacked = F.pad(torch.cat([p_hp, t_hp, p_hp**2, t_hp**2, p_hp * t_hp], 1), (lo, hi, lo, hi))
    m = F.conv2d(stacked, win.expand(5, 1, -1, -1), groups=5)
    mp, mt, epp, ett, ept = m.unbind(1)
    var_p = (epp - mp**2).clamp(min=0)
    var_t = (ett - mt**2).clamp(min=0)
    cov = ept - mt * mp
    den = torch.sqrt(var_t) * torch.sqrt(var_p)
    scc = torch.where(den == 0, torch.zeros_like(cov), cov / torch.where(den == 0, 1.0, den))
    return scc.reshape(b, c, *scc.shape[-2:])


def spatial_correlation_coefficient(
    preds: Tensor,
    target: Tensor,
    hp_filter: Optional[Tensor] = None,
    window_size: int = 8,
    reduction: Optional[Literal["mean", "none", None]] = "mean",
) -> Tensor:
    """Spatial correlation coefficient of high-pass filtered images."""
    if hp_filter is None:
        hp_filter = torch.tensor([[-1, -1, -1], [-1, 8, -1], [-1, -1, -1]])
    if reduction is None:
        reduction = "none"
    if reduction not in ("mean", "none"):
        raise ValueError(f"Expected reduction to be 'mean' or 'none', but got {reduction}")
    preds, target, hp_filter = _scc_update(preds, target, hp_filter, window_size)
    per_image = _scc_plane_means(preds, target, hp_filter, window_size)
    if reduction == "none":
        return per_image
    return per_image.mean()


# ------------------------------------------------------------------------------------------------------------ VIF
def _vif_filter(win_size: float, sigma: float, dtype: torch.dtype, device: torch.device) -> Tensor:
    coords = torch.arange(win_size, dtype=dtype, device=device) - (win_size - 1) / 2
    g = torch.exp(-(coords[None, :] ** 2 + coords[:, None] ** 2) / (2.0 * sigma**2))
    return g / g.sum()


def _vif_planes(preds: Tensor, target: Tensor, sigma_n_sq: float) -> Tensor:
    """Pixel-domain VIF of ``[P, 1, H, W]`` planes -> ``[P]``.

    ROCm: each scale's windowed moments and the per-window VIF terms are one launch of the SSIM window kernel in its
    VIF mode (separable Gaussian, valid windows, per-tile sums of numerator and denominator); only the 2x
    downsampling between scales stays a strided convolution.  The reference stacks 5 maps, runs a grouped conv and
    ~25 elementwise ops per scale (``F/image/vif.py:41-80``)."""
    if preds.is_cuda and preds.dtype in (torch.float32, torch.float64):
        return _vif_planes_fused(preds, target, sigma_n_sq)
    dtype, device = preds.dtype, preds.device
    eps = torch.tensor(1e-10, dtype=dtype, device=device)
    sn = torch.tensor(sigma_n_sq, dtype=dtype, device=device)
    num = torch.zeros(preds.shape[0], dtype=dtype, device=device)
    den = torch.zeros_like(num)
    for scale in range(4):
        n = 2.0 ** (4 - scale) + 1
        k = _vif_filter(n, n / 5, dtype, device)[None, None]
        if scale > 0:
            target = F.conv2d(target, k)[:, :, ::2, ::2]
            preds = F.conv2d(preds, k)[:, :, ::2, ::2]
        m = F.conv2d(torch.cat([target, preds, target**2, preds**2, target * preds], 1), k.expand(5, 1, -1, -1),
                     groups=5)
        mu_t, mu_p, e_tt, e_pp, e_tp = m.unbind(1)
        s_tt = torch.clamp(e_tt - mu_t**2, min=0.0)
        s_pp = torch.clamp(e_pp - mu_p**2, min=0.0)
        s_tp = e_tp - mu_t * mu_p
        g = s_tp / (s_tt + eps)
        s_v = s_pp - g * s_tp
        low_t = s_tt < eps
        g = torch.where(low_t, torch.zeros_like(g), g)
        s_v = torch.where(low_t, s_pp, s_v)
        s_tt = torch.where(low_t, torch.zeros_like(s_tt), s_tt)
        low_p = s_pp < eps
        g = torch.where(low_p, torch.zeros_like(g), g)
        s_v = torch.where(low_p, torch.zeros_like(s_v), s_v)
        neg = g < 0
        s_v = torch.where(neg, s_pp, s_v)
        g = torch.where(neg, torch.zeros_like(g), g)
        s_v = torch.clamp(s_v, min=eps)
        num = num + torch.log10(1.0 + g**2 * s_tt / (s_v + sn)).sum(dim=[1, 2])
        den = den + torch.log10(1.0 + s_tt / sn).sum(dim=[1, 2])
    return num / den


def _vif_planes_fused(preds: Tensor, target: Tensor, sigma_n_sq: float) -> Tensor:
    dtype, device = preds.dtype, preds.device
    consts = torch.tensor([sigma_n_sq, 0.0, 1e-10], dtype=dtype, device=device)
    num = torch.zeros(preds.shape[0], dtype=dtype, device=device)
    den = torch.zeros_like(num)
    for scale in range(4):
        n = 2.0 ** (4 - scale) + 1
        k2 = _vif_filter(n, n / 5, dtype, device)
        if scale > 0:
            target = F.conv2d(target, k2[None, None])[:, :, ::2, ::2]
            preds = F.conv2d(preds, k2[None, None])[:, :, ::2, ::2]
        k1 = k2.sum(1)  # the normalised 2-D Gaussian is the outer product of this 1-D one with itself
        part = ops.ssim2d_partials(target[:, 0].contiguous(), preds[:, 0].contiguous(), k1, k1, consts, ops.VIF_MODE)
        sums = part.sum(1)
        num = num + sums[:, 0].to(dtype)
        den = den + sums[:, 1].to(dtype)
    return num / den


def visual_information_fidelity(preds: Tensor, target: Tensor, sigma_n_sq: float = 2.0) -> Tensor:
    """Pixel-domain visual information fidelity (images at least 41 x 41)."""
    if preds.size(-1) < 41 or preds.size(-2) < 41:
        raise ValueError(f"Invalid size of preds. Expected at least 41x41, but got {preds.size(-1)}x{preds.size(-2)}!")
    if target.size(-1) < 41 or target.size(-2) < 41:
        raise ValueError(
            f"Invalid size of target. Expected at least 41x41, but got {target.size(-1)}x{target.size(-2)}!"
        )
    b, c, h, w = preds.shape
    # plane order channel-major to match the reference's per-channel concatenation
    p = preds.transpose(0, 1).reshape(c * b, 1, h, w)
    t = target.transpose(0, 1).reshape(c * b, 1, h, w)
    return _vif_planes(p, t, sigma_n_sq).mean()


# ------------------------------------------------------------------------------------------------------ D_lambda
def _spectral_distortion_index_update(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    if preds.dtype != target.dtype:
        raise TypeError(
            f"Expected `ms` and `fused` to have the same data type. Got ms: {preds.dtype} and fused: {target.dtype}."
        )
    if len(preds.shape) != 4:
        raise ValueError(
            f"Expected `preds` and `target` to have BxCxHxW shape. Got preds: {preds.shape} and target: {target.shape}."
        )
    if preds.shape[:2] != target.shape[:2]:
        raise ValueError(
            "Expected `preds` and `target` to have same batch and channel sizes."
            f"Got preds: {preds.shape} and target: {target.shape}."
        )
    return preds, target


def _band_uqi_matrix(x: Tensor) -> Tensor:
    """Symmetric ``[C, C]`` matrix of per-band-pair UQI (mean over the batch), all pairs in one batched call."""
    b, c = x.shape[:2]
    m = torch.zeros(c, c, dtype=x.dtype, device=x.device)
    if c < 2:
        return m
    iu = torch.triu_indices(c, c, offset=1, device=x.device)
    a = x[:, iu[0]].transpose(0, 1).reshape(-1, 1, *x.shape[-2:])  # [pairs*B, 1, H, W]
    bb = x[:, iu[1]].transpose(0, 1).reshape(-1, 1, *x.shape[-2:])
    per_pair = _uqi_plane_means(a, bb).reshape(iu.shape[1], -1).mean(1)
    m[iu[0], iu[1]] = per_pair.to(m.dtype)
    return m + m.T


def _spectral_distortion_index_compute(
    preds: Tensor, target: Tensor, p: int = 1,
    reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
) -> Tensor:
    length = preds.shape[1]
    m1, m2 = _band_uqi_matrix(target), _band_uqi_matrix(preds)
    diff = torch.pow(torch.abs(m1 - m2), p)
    if length == 1:
        out = torch.pow(diff, 1.0 / p)
    else:
        out = torch.pow(1.0 / (length * (length - 1)) * torch.sum(diff), 1.0 / p)
    return reduce(out, reduction)


def spectral_distortion_index(
    preds: Tensor, target: Tensor, p: int = 1,
    reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
) -> Tensor:
    """D_lambda: spectral distortion between the band-pair similarity structure of two images."""
    if not isinstance(p, int) or p <= 0:
        raise ValueError(f"Expected `p` to be a positive integer. Got p: {p}.")
    preds, target = _spectral_distortion_index_update(preds, target)
    return _spectral_distortion_index_compute(preds, target, p, reduction)


# ----------------------------------------------------------------------------------------------------------- D_s
def _spatial_distortion_index_update(
    preds: Tensor, ms: Tensor, pan: Tensor, pan_lr: Optional[Tensor] = None
) -> Tuple[Tensor, Tensor, Tensor, Optional[Tensor]]:
    for name, t in (("preds", preds), ("ms", ms), ("pan", pan)) + ((("pan_lr", pan_lr),) if pan_lr is not None else ()):
        if len(t.shape) != 4:
            raise ValueError(f"Expected `{name}` to have BxCxHxW shape. Got {name}: {t.shape}.")
        if t.dtype != preds.dtype:
            raise TypeError(
                f"Expected `preds` and `{name}` to have the same data type. Got preds: {preds.dtype} and {name}:"
                f" {t.dtype}."
            )
        if t.shape[:2] != preds.shape[:2]:
            raise ValueError(
                f"Expected `preds` and `{name}` to have the same batch and channel sizes."
                f" Got preds: {preds.shape} and {name}: {t.shape}."
            )
    (ph, pw), (mh, mw), (qh, qw) = preds.shape[-2:], ms.shape[-2:], pan.shape[-2:]
    if ph != qh:
        raise ValueError(f"Expected `preds` and `pan` to have the same height. Got preds: {ph} and pan: {qh}")
    if pw != qw:
        raise ValueError(f"Expected `preds` and `pan` to have the same width. Got preds: {pw} and pan: {qw}")
    if ph % mh != 0:
        raise ValueError(f"Expected height of `preds` to be multiple of height of `ms`. Got preds: {ph} and ms: {mh}.")
    if pw % mw != 0:
        raise ValueError(f"Expected width of `preds` to be multiple of width of `ms`. Got preds: {pw} and ms: {mw}.")
    if pan_lr is not None and pan_lr.shape[-2:] != ms.shape[-2:]:
        raise ValueError(
            f"Expected `ms` and `pan_lr` to have the same height and width. Got ms: {ms.shape} and pan_lr:"
            f" {pan_lr.shape}."
        )
    return preds, ms, pan, pan_lr


def _spatial_distortion_index_compute(
    preds: Tensor,
    ms: Tensor,
    pan: Tensor,
    pan_lr: Optional[Tensor] = None,
    norm_order: int = 1,
    window_size: int = 7,
    reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
) -> Tensor:
    ms_h, ms_w = ms.shape[-2:]
    if window_size >= ms_h or window_size >= ms_w:
        raise ValueError(
            f"Expected `window_size` to be smaller than dimension of `ms`. Got window_size: {window_size}."
        )
    if pan_lr is None:
        degraded = _uniform_filter(pan, window_size=window_size)
        pan_lr = F.interpolate(degraded, size=(ms_h, ms_w), mode="bilinear", align_corners=False, antialias=False)
    c = preds.shape[1]

    def per_band(a: Tensor, b: Tensor) -> Tensor:
        # UQI of each band over the batch: planes [C*B, 1, H, W], mean per band
        aa = a.transpose(0, 1).reshape(-1, 1, *a.shape[-2:])
        bb = b.transpose(0, 1).reshape(-1, 1, *b.shape[-2:])
        return _uqi_plane_means(aa, bb).reshape(c, -1).mean(1)

    m1, m2 = per_band(ms, pan_lr), per_band(preds, pan)
    diff = (m1 - m2).abs() ** norm_order
    return reduce(diff, reduction) ** (1 / norm_order)


def spatial_distortion_index(
    preds: Tensor,
    ms: Tensor,
    pan: Tensor,
    pan_lr: Optional[Tensor] = None,
    norm_order: int = 1,
    window_size: int = 7,
    reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
) -> Tensor:
    """D_s: spatial distortion of a pansharpened image w.r.t. the panchromatic band."""
    if not isinstance(norm_order, int) or norm_order <= 0:
        raise ValueError(f"Expected `norm_order` to be a positive integer. Got norm_order: {norm_order}.")
    if not isinstance(window_size, int) or window_size <= 0:
        raise ValueError(f"Expected `window_size` to be a positive integer. Got window_size: {window_size}.")
    preds, ms, pan, pan_lr = _spatial_distortion_index_update(preds, ms, pan, pan_lr)
    return _spatial_distortion_index_compute(preds, ms, pan, pan_lr, norm_order, window_size, reduction)


def quality_with_no_reference(
    preds: Tensor,
    ms: Tensor,
    pan: Tensor,
    pan_lr: Optional[Tensor] = None,
    alpha: float = 1,
    beta: float = 1,
    norm_order: int = 1,
    window_size: int = 7,
    reduction: Literal["elementwise_mean", "sum", "none"] = "elementwise_mean",
) -> Tensor:
    """QNR = (1 - D_lambda)^alpha * (1 - D_s)^beta."""
    if not isinstance(alpha, (int, float)) or alpha < 0:
        raise ValueError(f"Expected `alpha` to be a non-negative real number. Got alpha: {alpha}.")
    if not isinstance(beta, (int, float)) or beta < 0:
        raise ValueError(f"Expected `beta` to be a non-negative real number. Got beta: {beta}.")
    d_lambda = spectral_distortion_index(preds, ms, norm_order, reduction)
    d_s = spatial_distortion_index(preds, ms, pan, pan_lr, norm_order, window_size, reduction)
    return (1 - d_lambda) ** alpha * (1 - d_s) ** beta
