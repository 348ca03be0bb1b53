"""Signal-to-noise / distortion ratios (reference ``F/audio/snr.py``, ``F/audio/sdr.py``).

SDR solves the ``filter_length``-tap distortion filter per sample from FFT auto/cross-correlations; the symmetric
Toeplitz system goes to the Levinson kernel (:func:`torchmetrics_amd.ops.toeplitz_solve`, O(L^2) per sample on
ROCm) instead of a dense ``[B, L, L]`` LU solve.
"""
import math
from typing import Optional, Tuple

import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.checks import _check_same_shape
from torchmetrics_amd.utilities.prints import rank_zero_warn


def _fused(preds: Tensor, target: Tensor, scale_invariant: bool, zero_mean: bool, rows_from: int = -1,
           seg_dims: int = 1) -> Optional[Tensor]:
    """One-launch ROCm evaluation (``ops.snr_rows``) when no gradient is needed; None -> the ATen formula.

    Rows are the leading dims before ``rows_from``; each row's trailing dims are flattened, and zero-mean centring
    runs over the last ``seg_dims`` dims' worth of samples (1: per signal; SA-SDR centres per speaker)."""
    if not (preds.is_cuda and target.is_cuda and preds.dtype == target.dtype and preds.is_floating_point()
            and preds.numel() > 0 and preds.ndim >= 1):
        return None
    if torch.is_grad_enabled() and (preds.requires_grad or target.requires_grad):
        return None
    lead = preds.shape[:rows_from] if rows_from != -1 else preds.shape[:-1]
    rows = 1
    for d in lead:
        rows *= d
    length = preds.numel() // max(rows, 1)
    seg = preds.shape[-1] if seg_dims == 1 else length
    out = ops.snr_rows(preds.reshape(rows, length), target.reshape(rows, length), seg, scale_invariant, zero_mean,
                       torch.finfo(preds.dtype).eps)
    return out.reshape(lead)


def _zero_mean(preds: Tensor, target: Tensor) -> Tuple[Tensor, Tensor]:
    return preds - preds.mean(dim=-1, keepdim=True), target - target.mean(dim=-1, keepdim=True)


def signal_noise_ratio(preds: Tensor, target: Tensor, zero_mean: bool = False) -> Tensor:
    """SNR in dB per sample over the last dim (``F/audio/snr.py:22``)."""
    _check_same_shape(preds, target)
    fused = _fused(preds, target, False, zero_mean)
    if fused is not None:
        return fused
    eps = torch.finfo(preds.dtype).eps
    if zero_mean:
        preds, target = _zero_mean(preds, target)
    noise = target - preds
    return 10 * torch.log10((torch.sum(target**2, dim=-1) + eps) / (torch.sum(noise**2, dim=-1) + eps))


def scale_invariant_signal_distortion_ratio(preds: Tensor, target: Tensor, zero_mean: bool = False) -> Tensor:
    """SI-SDR in dB (``F/audio/sdr.py:211``)."""
    _check_same_shape(preds, target)
    fused = _fused(preds, target, True, zero_mean)
    if fused is not None:
        return fused
    eps = torch.finfo(preds.dtype).eps
    if zero_mean:
        preds, target = _zero_mean(preds, target)
    alpha = (torch.sum(preds * target, dim=-1, keepdim=True) + eps) / (torch.sum(target**2, dim=-1, keepdim=True) + eps)
    scaled = alpha * target
    noise = scaled - preds
    return 10 * torch.log10((torch.sum(scaled**2, dim=-1) + eps) / (torch.sum(noise**2, dim=-1) + eps))


def scale_invariant_signal_noise_ratio(preds: Tensor, target: Tensor) -> Tensor:
    """SI-SNR = zero-mean SI-SDR (``F/audio/snr.py:59``)."""
    return scale_invariant_signal_distortion_ratio(preds=preds, target=target, zero_mean=True)


def complex_scale_invariant_signal_noise_ratio(preds: Tensor, target: Tensor, zero_mean: bool = False) -> Tensor:
    """C-SI-SNR over ``(..., freq, time, 2)`` real or ``(..., freq, time)`` complex spectra (``F/audio/snr.py:84``)."""
    if preds.is_complex():
        preds = torch.view_as_real(preds)
    if target.is_complex():
        target = torch.view_as_real(target)
    if (preds.ndim < 3 or preds.shape[-1] != 2) or (target.ndim < 3 or target.shape[-1] != 2):
        raise RuntimeError(
            "Predictions and targets are expected to have the shape (..., frequency, time, 2),"
            f" but got {preds.shape} and {target.shape}."
        )
    preds = preds.reshape(*preds.shape[:-3], -1)
    target = target.reshape(*target.shape[:-3], -1)
    return scale_invariant_signal_distortion_ratio(preds=preds, target=target, zero_mean=zero_mean)


def _symmetric_toeplitz(vector: Tensor) -> Tensor:
    """``[..., L]`` -> the symmetric Toeplitz matrices ``[..., L, L]`` with first row ``vector`` (a strided view of
    the mirrored vector; reference ``F/audio/sdr.py:28``).  The SDR solve itself never forms this matrix: it runs
    the Levinson recursion on ``vector`` (:func:`torchmetrics_amd.ops.toeplitz_solve`)."""
    length = vector.shape[-1]
    mirrored = torch.cat([vector[..., 1:].flip(-1), vector], dim=-1)  # [v_{L-1} .. v_1, v_0 .. v_{L-1}]
    # window k of the mirrored vector is row L-1-k of the matrix
    return mirrored.unfold(-1, length, 1).flip(-2)


def _compute_autocorr_crosscorr(target: Tensor, preds: Tensor, corr_len: int) -> Tuple[Tensor, Tensor]:
    n_fft = 2 ** math.ceil(math.log2(preds.shape[-1] + target.shape[-1] - 1))
    t_fft = torch.fft.rfft(target, n=n_fft, dim=-1)
    r_0 = torch.fft.irfft(t_fft.real**2 + t_fft.imag**2, n=n_fft)[..., :corr_len]
    p_fft = torch.fft.rfft(preds, n=n_fft, dim=-1)
    b = torch.fft.irfft(t_fft.conj() * p_fft, n=n_fft, dim=-1)[..., :corr_len]
    return r_0, b


def signal_distortion_ratio(preds: Tensor, target: Tensor, use_cg_iter: Optional[int] = None,
                            filter_length: int = 512, zero_mean: bool = False,
                            load_diag: Optional[float] = None) -> Tensor:
    """SDR in dB with a ``filter_length``-tap allowed distortion filter (``F/audio/sdr.py:72``)."""
    _check_same_shape(preds, target)
    in_dtype = preds.dtype
    preds, target = preds.double(), target.double()
    if zero_mean:
        preds, target = _zero_mean(preds, target)
    target = target / torch.clamp(torch.linalg.norm(target, dim=-1, keepdim=True), min=1e-6)
    preds = preds / torch.clamp(torch.linalg.norm(preds, dim=-1, keepdim=True), min=1e-6)
    r_0, b = _compute_autocorr_crosscorr(target, preds, corr_len=filter_length)
    if load_diag is not None:
        r_0[..., 0] += load_diag
    if use_cg_iter is not None:
        rank_zero_warn(
            "The `use_cg_iter` parameter of `SDR` requires that `fast-bss-eval` is installed; the exact Toeplitz solver"
            " (Levinson on ROCm) is used instead.",
            UserWarning,
        )
    sol = ops.toeplitz_solve(r_0, b)
    coh = torch.einsum("...l,...l->...", b, sol)
    val = 10.0 * torch.log10(coh / (1 - coh))
    return val if in_dtype == torch.float64 else val.float()


def source_aggregated_signal_distortion_ratio(preds: Tensor, target: Tensor, scale_invariant: bool = True,
                                              zero_mean: bool = False) -> Tensor:
    """SA-SDR over ``(..., spk, time)`` (``F/audio/sdr.py:248``)."""
    _check_same_shape(preds, target)
    if preds.ndim < 2:
        raise RuntimeError(f"The preds and target should have the shape (..., spk, time), but {preds.shape} found")
    # one row per (...) item over (spk, time); zero_mean centres each speaker's signal
    fused = _fused(preds, target, scale_invariant, zero_mean, rows_from=-2, seg_dims=1)
    if fused is not None:
        return fused
    eps = torch.finfo(preds.dtype).eps
    if zero_mean:
        preds, target = _zero_mean(preds, target)
    if scale_invariant:
        alpha = ((preds * target).sum(dim=-1, keepdim=True).sum(dim=-2, keepdim=True) + eps) / (
            (target**2).sum(dim=-1, keepdim=True).sum(dim=-2, keepdim=True) + eps)
        target = alpha * target
    distortion = target - preds
    return 10 * torch.log10(((target**2).sum(dim=-1).sum(dim=-1) + eps) /
                            ((distortion**2).sum(dim=-1).sum(dim=-1) + eps))
