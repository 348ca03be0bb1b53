"""Speech-to-reverberation modulation energy ratio (reference ``F/audio/srmr.py``; SRMRpy algorithm).

The reference needs the ``gammatone`` and ``torchaudio`` packages for the cochlear filterbank design and ``lfilter``.
Here the filterbank is designed natively (Slaney's ERB-spaced 4th-order gammatone, as four cascaded biquads), and both
IIR stages (23 cochlear channels, then 8 modulation bands per channel) run in the fused cascade kernel
:func:`torchmetrics_amd.ops.biquad_cascade` (one thread per (signal, channel) row, all sections in registers).  The
FFT gammatonegram of ``fast=True`` still needs ``gammatone`` (``fft_gtgram``), like the reference.
"""
import math
from functools import lru_cache
from typing import Optional, Tuple

import numpy as np
import torch
from torch import Tensor
from torch.nn.functional import pad

from torchmetrics_amd import ops
from torchmetrics_amd.utilities.imports import _GAMMATONE_AVAILABLE
from torchmetrics_amd.utilities.prints import rank_zero_warn

_EAR_Q, _MIN_BW = 9.26449, 24.7  # Glasberg & Moore ERB parameters


def _centre_freqs(fs: int, num_freqs: int, cutoff: float) -> np.ndarray:
    """ERB-spaced centre frequencies from ``fs / 2`` down to ``cutoff`` (highest first)."""
    k = np.arange(1, num_freqs + 1)
    a = _EAR_Q * _MIN_BW
    return -a + np.exp(k * (-np.log(fs / 2 + a) + np.log(cutoff + a)) / num_freqs) * (fs / 2 + a)


def _calc_erbs(low_freq: float, fs: int, n_filters: int, device: torch.device) -> Tensor:
    return torch.tensor(_centre_freqs(fs, n_filters, low_freq) / _EAR_Q + _MIN_BW, device=device)


@lru_cache(maxsize=100)
def _make_erb_filters(fs: int, num_freqs: int, cutoff: float) -> np.ndarray:
    """``[num_freqs, 10]`` = (A0, A11, A12, A13, A14, A2, B0, B1, B2, gain) of the 4-stage gammatone cascade."""
    cf = _centre_freqs(fs, num_freqs, cutoff)
    t = 1.0 / fs
    erb = cf / _EAR_Q + _MIN_BW
    b = 1.019 * 2 * np.pi * erb
    arg = 2 * cf * np.pi * t
    eb = np.exp(b * t)
    a0, a2, b0 = t, 0.0, 1.0
    b1 = -2 * np.cos(arg) / eb
    b2 = np.exp(-2 * b * t)
    r_plus, r_minus = np.sqrt(3 + 2**1.5), np.sqrt(3 - 2**1.5)
    base = 2 * t * np.cos(arg) / eb
    a11 = -(base + 2 * r_plus * t * np.sin(arg) / eb) / 2
    a12 = -(base - 2 * r_plus * t * np.sin(arg) / eb) / 2
    a13 = -(base + 2 * r_minus * t * np.sin(arg) / eb) / 2
    a14 = -(base - 2 * r_minus * t * np.sin(arg) / eb) / 2
    z4, z2 = np.exp(4j * cf * np.pi * t), np.exp(-(b * t) + 2j * cf * np.pi * t)
    num = np.ones_like(z4)
    for sign, r in ((-1, r_minus), (1, r_minus), (-1, r_plus), (1, r_plus)):
        num = num * (-2 * z4 * t + 2 * z2 * t * (np.cos(arg) + sign * r * np.sin(arg)))
    den = (-2 / np.exp(2 * b * t) - 2 * z4 + 2 * (1 + z4) / eb) ** 4
    gain = np.abs(num / den)
    n = num_freqs
    return np.stack([np.full(n, a0), a11, a12, a13, a14, np.full(n, a2), np.full(n, b0), b1, b2, gain], axis=1)


def _gammatone_sections(fcoefs: np.ndarray) -> np.ndarray:
    """``[F, 4, 6]`` biquads: shared denominator (B0, B1, B2), numerators (A0, A1k, A2)."""
    sec = np.zeros((fcoefs.shape[0], 4, 6))
    for s, col in enumerate((1, 2, 3, 4)):
        sec[:, s, 0] = fcoefs[:, 0]
        sec[:, s, 1] = fcoefs[:, col]
        sec[:, s, 2] = fcoefs[:, 5]
        sec[:, s, 3:6] = fcoefs[:, 6:9]
    return sec


@lru_cache(maxsize=100)
def _compute_modulation_filterbank_and_cutoffs(min_cf: float, max_cf: float, n: int, fs: float,
                                               q: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Log-spaced Q=2 second-order band-pass modulation filters: (centres, [n, 2, 3] (b, a), low / high 3 dB)."""
    cfs = min_cf * (max_cf / min_cf) ** (np.arange(n) / (n - 1))
    w0 = np.tan(np.pi * cfs / fs)  # tan(w / 2) with w = 2 pi cf / fs
    b0 = w0 / q
    b = np.stack([b0, np.zeros(n), -b0], axis=1)
    a = np.stack([1 + b0 + w0**2, 2 * w0**2 - 2, 1 - b0 + w0**2], axis=1)
    half_bw = np.tan(np.pi * cfs / fs) / q * fs / (2 * np.pi)
    return cfs, np.stack([b, a], axis=1), cfs - half_bw, cfs + half_bw


def _hilbert(x: Tensor, n: Optional[int] = None) -> Tensor:
    """Analytic signal via the FFT (length rounded up to a multiple of 16)."""
    if x.is_complex():
        raise ValueError("x must be real.")
    if n is None:
        n = x.shape[-1]
        if n % 16:
            n = math.ceil(n / 16) * 16
    if n <= 0:
        raise ValueError("N must be positive.")
    h = torch.zeros(n, dtype=x.dtype, device=x.device)
    if n % 2 == 0:
        h[0] = h[n // 2] = 1
        h[1 : n // 2] = 2
    else:
        h[0] = 1
        h[1 : (n + 1) // 2] = 2
    return torch.fft.ifft(torch.fft.fft(x, n=n, dim=-1) * h, dim=-1)[..., : x.shape[-1]]


def _normalize_energy(energy: Tensor, drange: float = 30.0) -> Tensor:
    peak = torch.mean(energy, dim=1, keepdim=True).amax(dim=2, keepdim=True).amax(dim=3, keepdim=True)
    low = peak * 10.0 ** (-drange / 10.0)
    return torch.minimum(torch.maximum(energy, low), peak)


def _srmr_arg_validate(fs: int, n_cochlear_filters: int = 23, low_freq: float = 125, min_cf: float = 4,
                       max_cf: Optional[float] = 128, norm: bool = False, fast: bool = False) -> None:
    if not (isinstance(fs, int) and fs > 0):
        raise ValueError(f"Expected argument `fs` to be an int larger than 0, but got {fs}")
    if not (isinstance(n_cochlear_filters, int) and n_cochlear_filters > 0):
        raise ValueError(
            f"Expected argument `n_cochlear_filters` to be an int larger than 0, but got {n_cochlear_filters}")
    if not (isinstance(low_freq, (float, int)) and low_freq > 0):
        raise ValueError(f"Expected argument `low_freq` to be a float larger than 0, but got {low_freq}")
    if not (isinstance(min_cf, (float, int)) and min_cf > 0):
        raise ValueError(f"Expected argument `min_cf` to be a float larger than 0, but got {min_cf}")
    if max_cf is not None and not (isinstance(max_cf, (float, int)) and max_cf > 0):
        raise ValueError(f"Expected argument `max_cf` to be a float larger than 0, but got {max_cf}")
    if not isinstance(norm, bool):
        raise ValueError("Expected argument `norm` to be a bool value")
    if not isinstance(fast, bool):
        raise ValueError("Expected argument `fast` to be a bool value")


def speech_reverberation_modulation_energy_ratio(preds: Tensor, fs: int, n_cochlear_filters: int = 23,
                                                 low_freq: float = 125, min_cf: float = 4,
                                                 max_cf: Optional[float] = None, norm: bool = False,
                                                 fast: bool = False) -> Tensor:
    """SRMR per signal of ``preds [..., time]`` (``F/audio/srmr.py:177``)."""
    _srmr_arg_validate(fs, n_cochlear_filters, low_freq, min_cf, max_cf, norm, fast)
    shape = preds.shape
    preds = preds.reshape(1, -1) if len(shape) == 1 else preds.reshape(-1, shape[-1])
    num_batch, time = preds.shape
    if not torch.is_floating_point(preds):
        preds = preds.to(torch.float64) / torch.finfo(preds.dtype).max
    max_vals = preds.abs().amax(dim=-1, keepdim=True)
    preds = preds / torch.where(max_vals > 1, max_vals, torch.ones_like(max_vals))
    dev = preds.device
    if fast:
        if not _GAMMATONE_AVAILABLE:
            raise ModuleNotFoundError("`fast=True` (FFT gammatonegram) requires the `gammatone` package.")
        from gammatone.fftweight import fft_gtgram

        rank_zero_warn("`fast=True` may slow down the speed of SRMR metric on GPU.")
        mfs = 400.0
        arr = preds.detach().cpu().numpy()
        gt_env = torch.stack([torch.tensor(fft_gtgram(arr[b], fs, 0.010, 0.0025, n_cochlear_filters, low_freq))
                              for b in range(num_batch)]).to(dev)
    else:
        fcoefs = _make_erb_filters(fs, n_cochlear_filters, float(low_freq))
        sections = torch.from_numpy(_gammatone_sections(fcoefs))
        y = ops.biquad_cascade(preds.double(), sections, rep=n_cochlear_filters, clamp=True)
        gain = torch.from_numpy(fcoefs[:, 9]).to(dev)
        y = y.reshape(num_batch, n_cochlear_filters, time) / gain.reshape(1, -1, 1)
        gt_env = torch.abs(_hilbert(y))  # [B, N, T]
        mfs = fs
    w_length = math.ceil(0.256 * mfs)
    w_inc = math.ceil(0.064 * mfs)
    if max_cf is None:
        max_cf = 30 if norm else 128
    _, mf, cutoffs, _ = _compute_modulation_filterbank_and_cutoffs(float(min_cf), float(max_cf), 8, float(mfs), 2)
    n_t = gt_env.shape[-1]
    num_frames = int(1 + (n_t - w_length) // w_inc)
    w = torch.hamming_window(w_length + 1, dtype=torch.float64, device=dev)[:-1]
    mod_sections = torch.from_numpy(np.concatenate([mf[:, 0, :], mf[:, 1, :]], axis=1)[:, None, :])  # [8, 1, 6]
    mod = ops.biquad_cascade(gt_env.reshape(-1, n_t).double(), mod_sections, rep=8, clamp=False)
    mod = mod.reshape(num_batch, n_cochlear_filters, 8, n_t)
    padding = (0, max(math.ceil(n_t / w_inc) * w_inc - n_t, w_length - n_t))
    frames = pad(mod, pad=padding, mode="constant", value=0).unfold(-1, w_length, w_inc)
    energy = ((frames[..., :num_frames, :] * w) ** 2).sum(dim=-1)  # [B, N, 8, frames]
    if norm:
        energy = _normalize_energy(energy)
    erbs = torch.flipud(_calc_erbs(low_freq, fs, n_cochlear_filters, dev))
    avg_energy = energy.mean(dim=-1)  # [B, N, 8]
    total = avg_energy.reshape(num_batch, -1).sum(-1)
    ac_perc = avg_energy.sum(dim=2) * 100 / total.reshape(-1, 1)
    ac_cum = ac_perc.flip(-1).cumsum(-1)
    k90 = torch.nonzero((ac_cum > 90).cumsum(-1) == 1)[:, 1]
    bw = erbs[k90]
    cut = torch.tensor(cutoffs, device=dev)
    scores = []
    for b in range(num_batch):
        if cut[4] <= bw[b] < cut[5]:
            kstar = 5
        elif cut[5] <= bw[b] < cut[6]:
            kstar = 6
        elif cut[6] <= bw[b] < cut[7]:
            kstar = 7
        elif cut[7] <= bw[b]:
            kstar = 8
        else:
            raise ValueError("Something wrong with the cutoffs compared to bw values.")
        scores.append(avg_energy[b, :, :4].sum() / avg_energy[b, :, 4:kstar].sum())
    score = torch.stack(scores)
    return score.reshape(*shape[:-1]) if len(shape) > 1 else score
