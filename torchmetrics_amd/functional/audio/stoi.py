"""Short-Time Objective Intelligibility (STOI) and extended STOI, native (reference ``F/audio/stoi.py:25``).

The reference calls the ``pystoi`` package per sample on the host (NumPy).  This is the same published algorithm
(Taal et al. 2011; Jensen & Taal 2016 for the extended variant) written for batched device execution:

1. resample to 10 kHz with the Octave-compatible Kaiser-windowed polyphase filter (``resample_poly`` semantics,
   computed as ONE strided ``conv1d`` over the zero-stuffed signals of the whole batch);
2. silent-frame removal: 256-sample Hann frames with hop 128, frames more than 40 dB below the loudest clean frame
   dropped, the kept frames overlap-added back (per signal: the kept-frame count is data dependent);
3. 512-point FFT of the frames (rocFFT on ROCm), one-third-octave band energies (15 bands from 150 Hz) by a
   ``[15, 257]`` band matrix product;
4. 30-frame sliding segments, clipping + normalisation and correlation, averaged over bands/segments: on ROCm one
   kernel over every segment of the batch (``csrc/audio/stoi.hip``, fp64, envelope windows staged in LDS), on the
   host ``unfold`` + tensor ops.

Steps 3-4 run for all signals at once, padded to the longest kept length and masked.  Signals with fewer than 30
kept frames return 1e-5 with a ``RuntimeWarning``, as pystoi does.  The extended variant's row/column normalisation
omits pystoi's 1e-16-scale random dither (deterministic here).  Parity status: the resampler is checked against
``scipy.signal.resample_poly`` and the pipeline against a NumPy transcription of the published algorithm
(``tests/test_audio.py``); ``pystoi`` itself and the reference's wav fixtures are not available, so the end-to-end
agreement with pystoi is unpinned.
"""
import math
import warnings
from functools import lru_cache
from typing import List, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor

from torchmetrics_amd.utilities.checks import _check_same_shape

FS = 10000
N_FRAME = 256
NFFT = 512
NUMBAND = 15
MINFREQ = 150
N_SEG = 30
BETA = -15.0
DYN_RANGE = 40.0
EPS = float(np.finfo(np.float64).eps)
_SHORT_MSG = ("Not enough STFT frames to compute intermediate intelligibility measure after removing silent frames."
              " Returning 1e-5. Please check you wav files")


@lru_cache(maxsize=None)
def _third_octave_matrix(fs: int = FS, nfft: int = NFFT, num_bands: int = NUMBAND,
                         min_freq: float = MINFREQ) -> np.ndarray:
    """One-third-octave band matrix ``[num_bands, nfft // 2 + 1]``: band edges snapped to the nearest FFT bin."""
    f = np.linspace(0, fs, nfft + 1)[: nfft // 2 + 1]
    k = np.arange(num_bands, dtype=np.float64)
    freq_low = min_freq * np.power(2.0, (2 * k - 1) / 6)
    freq_high = min_freq * np.power(2.0, (2 * k + 1) / 6)
    obm = np.zeros((num_bands, len(f)))
    for i in range(num_bands):
        lo = int(np.argmin(np.square(f - freq_low[i])))
        hi = int(np.argmin(np.square(f - freq_high[i])))
        obm[i, lo:hi] = 1.0
    return obm


@lru_cache(maxsize=None)
def _octave_resample_filter(p: int, q: int) -> Tuple[np.ndarray, int, int]:
    """Kaiser-windowed sinc of Octave's ``resample`` (60 dB rejection) for a ``p / q`` rate change, normalised to
    unit DC gain; returns ``(h, p, q)`` with ``p / q`` reduced."""
    g = math.gcd(p, q)
    p, q = p // g, q // g
    log10_rejection = -3.0
    stopband_cutoff_f = 1.0 / (2 * max(p, q))
    roll_off_width = stopband_cutoff_f / 10
    rejection_db = -20 * log10_rejection
    half = int(np.ceil((rejection_db - 8) / (28.714 * roll_off_width)))
    t = np.arange(-half, half + 1)
    ideal = 2 * p * stopband_cutoff_f * np.sinc(2 * stopband_cutoff_f * t)
    if 21 <= rejection_db <= 50:
        beta = 0.5842 * (rejection_db - 21) ** 0.4 + 0.07886 * (rejection_db - 21)
    elif rejection_db > 50:
        beta = 0.1102 * (rejection_db - 8.7)
    else:
        beta = 0.0
    h = np.kaiser(2 * half + 1, beta) * ideal
    return h / np.sum(h), p, q


def _resample_poly(x: Tensor, up: int, down: int, window: np.ndarray) -> Tensor:
    """``scipy.signal.resample_poly(x, up, down, window=window)`` along the last dim of ``[B, T]``.

    Zero-stuff by ``up``, FIR filter (``window * up``), keep every ``down``-th sample with scipy's centring offsets;
    the filtering and the decimation are one ``conv1d`` with ``stride = down``."""
    b, n_in = x.shape
    h = torch.as_tensor(window * up, dtype=x.dtype, device=x.device)
    half_len = (h.numel() - 1) // 2
    n_out = n_in * up // down + int(n_in * up % down != 0)
    n_pre_pad = down - half_len % down
    n_pre_remove = (half_len + n_pre_pad) // down
    h_len = h.numel() + n_pre_pad
    n_post_pad = 0  # as scipy: extend the filter until the upfirdn output covers the kept samples
    while ((n_in - 1) * up + h_len + n_post_pad - 1) // down + 1 < n_out + n_pre_remove:
        n_post_pad += 1
    h = torch.cat([h.new_zeros(n_pre_pad), h, h.new_zeros(n_post_pad)])
    up_x = x.new_zeros(b, n_in * up)
    up_x[:, ::up] = x
    # full convolution z[m] = sum_k h[k] x_up[m - k]; only m = (n_pre_remove + j) * down is evaluated
    k = h.numel()
    padded = F.pad(up_x, (k - 1, k - 1))
    first = n_pre_remove * down
    y = F.conv1d(padded[:, None, first:], h.flip(0)[None, None, :], stride=down)[:, 0]
    return y[:, :n_out]


def _frames(x: Tensor, framelen: int, hop: int) -> Tensor:
    """Hann-windowed frames ``[B, F, framelen]`` starting at ``range(0, T - framelen, hop)`` (pystoi's grid)."""
    count = len(range(0, x.shape[-1] - framelen, hop))
    w = torch.hann_window(framelen + 2, periodic=False, dtype=x.dtype, device=x.device)[1:-1]
    if count == 0:
        return x.new_zeros(x.shape[0], 0, framelen)
    return x.unfold(-1, framelen, hop)[:, :count] * w


def _overlap_add(frames: Tensor, hop: int) -> Tensor:
    """Plain overlap-add of ``[F, framelen]`` frames at stride ``hop`` (length ``(F - 1) * hop + framelen``)."""
    nf, framelen = frames.shape
    out = frames.new_zeros((nf - 1) * hop + framelen)
    pos = torch.arange(nf, device=frames.device)[:, None] * hop + torch.arange(framelen, device=frames.device)[None]
    out.index_put_((pos.reshape(-1),), frames.reshape(-1), accumulate=True)
    return out


def _remove_silent_frames(x: Tensor, y: Tensor) -> Tuple[List[Tensor], List[Tensor]]:
    """Per signal: drop frames more than 40 dB below the loudest clean frame, overlap-add the rest."""
    hop = N_FRAME // 2
    xf, yf = _frames(x, N_FRAME, hop), _frames(y, N_FRAME, hop)
    energies = 20 * torch.log10(torch.linalg.norm(xf, dim=-1) + EPS)
    keep = (energies.max(dim=-1, keepdim=True).values - DYN_RANGE - energies) < 0
    xs, ys = [], []
    for i in range(x.shape[0]):  # the kept-frame count is data dependent per signal
        xs.append(_overlap_add(xf[i][keep[i]], hop))
        ys.append(_overlap_add(yf[i][keep[i]], hop))
    return xs, ys


def _band_envelopes(sig: Tensor) -> Tensor:
    """``[B, 15, frames]`` one-third-octave band magnitudes of ``[B, T]`` signals."""
    fr = _frames(sig, N_FRAME, N_FRAME // 2)
    spec = torch.fft.rfft(fr, n=NFFT, dim=-1)  # [B, F, 257]
    obm = torch.as_tensor(_third_octave_matrix(), dtype=sig.dtype, device=sig.device)
    return torch.sqrt(torch.matmul(spec.abs().square(), obm.t())).transpose(1, 2)


def _stoi_batch(x: Tensor, y: Tensor, extended: bool) -> Tensor:
    """STOI of clean ``x`` vs processed ``y``, both ``[B, T]`` at 10 kHz."""
    if x.shape[-1] <= N_FRAME:
        warnings.warn(_SHORT_MSG, RuntimeWarning)
        return torch.full((x.shape[0],), 1e-5, dtype=x.dtype, device=x.device)
    xs, ys = _remove_silent_frames(x, y)
    lens = [t.numel() for t in xs]
    longest = max(lens)
    xp = torch.stack([F.pad(t, (0, longest - t.numel())) for t in xs])
    yp = torch.stack([F.pad(t, (0, longest - t.numel())) for t in ys])
    n_frames = torch.tensor([len(range(0, n - N_FRAME, N_FRAME // 2)) for n in lens], device=x.device)
    short_val = torch.full((x.shape[0],), 1e-5, dtype=x.dtype, device=x.device)
    x_tob, y_tob = _band_envelopes(xp), _band_envelopes(yp)  # [B, J, frames]
    if x_tob.shape[-1] < N_SEG:
        warnings.warn(_SHORT_MSG, RuntimeWarning)
        return short_val
    m_valid = (n_frames - N_SEG + 1).clamp(min=0)  # segments entirely inside each signal's kept frames
    short = m_valid < 1
    if x_tob.is_cuda:
        # every segment of every signal in one launch, fp64, windows staged in LDS (csrc/audio/stoi.hip)
        from torchmetrics_amd import ops

        sums = ops.stoi_segments(x_tob, y_tob, n_frames, extended)
        vals = (sums / (m_valid.clamp(min=1) * (1 if extended else NUMBAND))).to(x.dtype)
        if bool(short.any()):
            warnings.warn(_SHORT_MSG, RuntimeWarning)
        return torch.where(short, short_val, vals)
    xseg = x_tob.unfold(-1, N_SEG, 1).transpose(1, 2)  # [B, M, J, N]
    yseg = y_tob.unfold(-1, N_SEG, 1).transpose(1, 2)
    seg_mask = (torch.arange(xseg.shape[1], device=x.device)[None, :] < m_valid[:, None]).to(x.dtype)
    if extended:
        def _unit(s: Tensor, dim: int) -> Tensor:
            s = s - s.mean(dim=dim, keepdim=True)
            n = torch.sqrt(torch.sum(s * s, dim=dim, keepdim=True))
            # an all-constant row/column has no direction: 0 here (pystoi dithers it with 1e-16 noise instead)
            return torch.where(n > 0, s / torch.where(n > 0, n, torch.ones_like(n)), torch.zeros_like(s))

        def _norm(s: Tensor) -> Tensor:  # rows (frames), then columns (bands)
            return _unit(_unit(s, -1), -2)

        corr = (_norm(xseg) * _norm(yseg) / N_SEG).sum(dim=(-1, -2))  # [B, M]
        vals = torch.where(seg_mask > 0, corr, torch.zeros_like(corr)).sum(-1) / m_valid.clamp(min=1)
    else:
        norm_const = torch.linalg.norm(xseg, dim=-1, keepdim=True) / (
            torch.linalg.norm(yseg, dim=-1, keepdim=True) + EPS)
        clip = 10 ** (-BETA / 20)
        y_primes = torch.minimum(yseg * norm_const, xseg * (1 + clip))
        y_primes = y_primes - y_primes.mean(dim=-1, keepdim=True)
        xc = xseg - xseg.mean(dim=-1, keepdim=True)
        y_primes = y_primes / (torch.linalg.norm(y_primes, dim=-1, keepdim=True) + EPS)
        xc = xc / (torch.linalg.norm(xc, dim=-1, keepdim=True) + EPS)
        corr = (y_primes * xc).sum(dim=(-1, -2))  # [B, M]
        vals = torch.where(seg_mask > 0, corr, torch.zeros_like(corr)).sum(-1) / (m_valid.clamp(min=1) * NUMBAND)
    if bool(short.any()):
        warnings.warn(_SHORT_MSG, RuntimeWarning)
    return torch.where(short, short_val, vals)


def short_time_objective_intelligibility(preds: Tensor, target: Tensor, fs: int, extended: bool = False,
                                         keep_same_device: bool = False) -> Tensor:
    """STOI (``extended=False``) or ESTOI per signal; ``preds`` / ``target`` are ``[..., time]``.

    Computed in float64 on the input's device; returns a float64 tensor of shape ``preds.shape[:-1]`` on the CPU
    unless ``keep_same_device`` (the reference's contract: its NumPy backend runs on the host)."""
    _check_same_shape(preds, target)
    if not isinstance(fs, int) or fs <= 0:
        raise ValueError(f"Expected argument `fs` to be a positive integer, but got {fs}")
    shape = preds.shape[:-1]
    x = target.detach().reshape(-1, target.shape[-1]).double()
    y = preds.detach().reshape(-1, preds.shape[-1]).double()
    if fs != FS:
        h, up, down = _octave_resample_filter(FS, fs)
        x = _resample_poly(x, up, down, h)
        y = _resample_poly(y, up, down, h)
    val = _stoi_batch(x, y, extended).reshape(shape)
    return val.to(preds.device) if keep_same_device else val.cpu()
