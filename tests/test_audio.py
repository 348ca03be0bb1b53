"""Audio metrics (reference ``tests/unittests/audio``).  mir_eval / fast_bss_eval / pesq / pystoi are not installed:
SNR-family values are pinned to the reference docstrings, SDR to a direct numpy least-squares oracle of the
distortion-filter projection and to the reference docstring values."""
import math

import numpy as np
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.audio import (
    ComplexScaleInvariantSignalNoiseRatio,
    PerceptualEvaluationSpeechQuality,
    PermutationInvariantTraining,
    ScaleInvariantSignalDistortionRatio,
    ScaleInvariantSignalNoiseRatio,
    ShortTimeObjectiveIntelligibility,
    SignalDistortionRatio,
    SignalNoiseRatio,
    SourceAggregatedSignalDistortionRatio,
)
from torchmetrics_amd.functional.audio import (
    complex_scale_invariant_signal_noise_ratio,
    permutation_invariant_training,
    pit_permutate,
    scale_invariant_signal_distortion_ratio,
    scale_invariant_signal_noise_ratio,
    short_time_objective_intelligibility,
    signal_distortion_ratio,
    signal_noise_ratio,
    source_aggregated_signal_distortion_ratio,
)

T = torch.tensor([3.0, -0.5, 2.0, 7.0])
P = torch.tensor([2.5, 0.0, 2.0, 8.0])


def test_docstring_values():
    assert torch.isclose(signal_noise_ratio(P, T), torch.tensor(16.1805), atol=1e-4)
    assert torch.isclose(scale_invariant_signal_noise_ratio(P, T), torch.tensor(15.0918), atol=1e-4)
    assert torch.isclose(scale_invariant_signal_distortion_ratio(P, T), torch.tensor(18.4030), atol=1e-4)
    torch.manual_seed(1)
    p, t = torch.randn((1, 257, 100, 2)), torch.randn((1, 257, 100, 2))
    assert torch.isclose(complex_scale_invariant_signal_noise_ratio(p, t), torch.tensor([-63.4849]), atol=1e-3)
    torch.manual_seed(1)
    p, t = torch.randn(8000), torch.randn(8000)
    assert torch.isclose(signal_distortion_ratio(p, t), torch.tensor(-12.0589), atol=1e-3)
    p, t = torch.randn(4, 2, 8000), torch.randn(4, 2, 8000)
    best, perm = permutation_invariant_training(p, t, signal_distortion_ratio)
    assert torch.allclose(best, torch.tensor([-11.6375, -11.4358, -11.7148, -11.6325]), atol=1e-3)
    assert perm.tolist() == [[1, 0], [0, 1], [1, 0], [0, 1]]
    torch.manual_seed(1)
    p, t = torch.randn(2, 8000), torch.randn(2, 8000)
    assert torch.isclose(source_aggregated_signal_distortion_ratio(p, t), torch.tensor(-41.6579), atol=1e-3)
    p, t = torch.randn(4, 2, 8000), torch.randn(4, 2, 8000)
    best, perm = permutation_invariant_training(p, t, source_aggregated_signal_distortion_ratio,
                                                mode="permutation-wise")
    assert torch.allclose(best, torch.tensor([-37.9511, -41.9124, -42.7369, -42.5155]), atol=1e-3)
    assert perm.tolist() == [[1, 0], [1, 0], [0, 1], [1, 0]]
    p = torch.tensor([[[-0.0579, 0.3560, -0.9604], [-0.1719, 0.3205, 0.2951]]])
    t = torch.tensor([[[1.0958, -0.1648, 0.5228], [-0.4100, 1.1942, -0.5103]]])
    best, perm = permutation_invariant_training(p, t, scale_invariant_signal_distortion_ratio,
                                                mode="speaker-wise", eval_func="max")
    assert torch.allclose(best, torch.tensor([-5.1091]), atol=1e-4) and perm.tolist() == [[0, 1]]
    assert torch.equal(pit_permutate(p, perm), p)


def _sdr_oracle(p, t, L=512):
    """Project normalised preds onto the span of L shifts of the normalised target (dense least squares)."""
    p = np.asarray(p, dtype=np.float64)
    t = np.asarray(t, dtype=np.float64)
    t = t / max(np.linalg.norm(t), 1e-6)
    p = p / max(np.linalg.norm(p), 1e-6)
    n = len(t)
    A = np.zeros((n + L - 1, L))
    for k in range(L):
        A[k:k + n, k] = t
    pp = np.concatenate([p, np.zeros(L - 1)])
    h, *_ = np.linalg.lstsq(A, pp, rcond=None)
    proj = A @ h
    coh = proj @ pp
    return 10 * np.log10(coh / (1 - coh))


def test_sdr_oracle_and_toeplitz():
    g = torch.Generator().manual_seed(3)
    t = torch.randn(3, 1000, generator=g)
    p = t + 0.5 * torch.randn(3, 1000, generator=g)
    got = signal_distortion_ratio(p, t, filter_length=64)
    ref = [_sdr_oracle(p[i], t[i], 64) for i in range(3)]
    assert np.allclose(got.numpy(), ref, atol=1e-3)
    r = torch.tensor([4.0, 1.0, 0.5, 0.25], dtype=torch.float64)
    b = torch.tensor([1.0, 2.0, 3.0, 4.0], dtype=torch.float64)
    x = ops.toeplitz_solve(r, b)
    from torchmetrics_amd.ops._cpu import symmetric_toeplitz

    assert torch.allclose(symmetric_toeplitz(r) @ x, b)


@pytest.mark.parametrize(
    ("cls", "fn", "kw"),
    [
        (SignalNoiseRatio, signal_noise_ratio, {"zero_mean": True}),
        (ScaleInvariantSignalNoiseRatio, scale_invariant_signal_noise_ratio, {}),
        (ScaleInvariantSignalDistortionRatio, scale_invariant_signal_distortion_ratio, {}),
        (SignalDistortionRatio, signal_distortion_ratio, {"filter_length": 32}),
        (SourceAggregatedSignalDistortionRatio, source_aggregated_signal_distortion_ratio, {}),
    ],
)
def test_modules_mean_of_batches(cls, fn, kw, device="cpu"):
    g = torch.Generator().manual_seed(0)
    batches = [(torch.randn(4, 2, 500, generator=g), torch.randn(4, 2, 500, generator=g)) for _ in range(3)]
    m = cls(**kw).to(device)
    vals = []
    for p, t in batches:
        m.update(p.to(device), t.to(device))
        vals.append(fn(p, t, **kw).reshape(-1))
    assert torch.allclose(m.compute().cpu().float(), torch.cat(vals).mean().float(), atol=1e-4)


def test_complex_and_pit_modules():
    g = torch.Generator().manual_seed(1)
    p, t = torch.randn(2, 17, 9, 2, generator=g), torch.randn(2, 17, 9, 2, generator=g)
    m = ComplexScaleInvariantSignalNoiseRatio()
    m.update(p, t)
    assert torch.isclose(m.compute(), complex_scale_invariant_signal_noise_ratio(p, t).mean())
    assert "num" in m._defaults and "ci_snr_sum" in m._defaults
    pit = PermutationInvariantTraining(scale_invariant_signal_distortion_ratio, eval_func="max")
    p, t = torch.randn(3, 3, 200, generator=g), torch.randn(3, 3, 200, generator=g)
    pit.update(p, t)
    best, _ = permutation_invariant_training(p, t, scale_invariant_signal_distortion_ratio)
    assert torch.isclose(pit.compute(), best.mean())


def test_pit_exhaustive_matches_assignment():
    """Device exhaustive search and scipy's Hungarian agree (4 speakers, random metric matrices)."""
    from torchmetrics_amd.functional.audio.pit import (
        _find_best_perm_by_exhaustive_method,
        _find_best_perm_by_linear_sum_assignment,
    )

    mm = torch.randn(16, 4, 4, generator=torch.Generator().manual_seed(2))
    for op in (torch.max, torch.min):
        a, pa = _find_best_perm_by_exhaustive_method(mm, op)
        b, pb = _find_best_perm_by_linear_sum_assignment(mm, op)
        assert torch.allclose(a, b) and torch.equal(pa, pb)


def test_external_wrappers_gated():
    with pytest.raises(ModuleNotFoundError):
        PerceptualEvaluationSpeechQuality(16000, "wb")


# ---------------------------------------------------------------------------------------------------------- STOI
# A NumPy transcription of the published STOI / ESTOI algorithm as pystoi implements it (frame grid, silent-frame
# removal, 1/3-octave bands, 30-frame segments, clipping at -15 dB SDR) -- pystoi itself is not installed, so this
# is the oracle; the resampler is checked against scipy.signal.resample_poly separately.
def _np_stoi(x, y, fs, extended):
    import scipy.signal

    from torchmetrics_amd.functional.audio import stoi as S

    if fs != S.FS:
        h, up, down = S._octave_resample_filter(S.FS, fs)
        x = scipy.signal.resample_poly(x, up, down, window=h)
        y = scipy.signal.resample_poly(y, up, down, window=h)
    eps = np.finfo("float").eps
    w = np.hanning(S.N_FRAME + 2)[1:-1]
    hop = S.N_FRAME // 2
    xf = np.array([w * x[i:i + S.N_FRAME] for i in range(0, len(x) - S.N_FRAME, hop)])
    yf = np.array([w * y[i:i + S.N_FRAME] for i in range(0, len(x) - S.N_FRAME, hop)])
    en = 20 * np.log10(np.linalg.norm(xf, axis=1) + eps)
    mask = (np.max(en) - S.DYN_RANGE - en) < 0
    xf, yf = xf[mask], yf[mask]

    def ola(fr):
        out = np.zeros((len(fr) - 1) * hop + S.N_FRAME)
        for i, f in enumerate(fr):
            out[i * hop:i * hop + S.N_FRAME] += f
        return out

    x, y = ola(xf), ola(yf)

    def spec(sig):
        return np.array([np.fft.rfft(w * sig[i:i + S.N_FRAME], n=S.NFFT)
                         for i in range(0, len(sig) - S.N_FRAME, hop)]).T

    xs, ys = spec(x), spec(y)
    if xs.shape[-1] < S.N_SEG:
        return 1e-5
    obm = S._third_octave_matrix()
    xt = np.sqrt(obm @ np.abs(xs) ** 2)
    yt = np.sqrt(obm @ np.abs(ys) ** 2)
    xseg = np.array([xt[:, m - S.N_SEG:m] for m in range(S.N_SEG, xt.shape[1] + 1)])
    yseg = np.array([yt[:, m - S.N_SEG:m] for m in range(S.N_SEG, xt.shape[1] + 1)])
    if extended:
        def rc(a):
            a = a - a.mean(-1, keepdims=True)
            a = a / np.sqrt((a ** 2).sum(-1, keepdims=True))
            a = a - a.mean(1, keepdims=True)
            return a / np.sqrt((a ** 2).sum(1, keepdims=True))

        xn, yn = rc(xseg), rc(yseg)
        return np.sum(xn * yn / S.N_SEG) / xn.shape[0]
    nc = np.linalg.norm(xseg, axis=2, keepdims=True) / (np.linalg.norm(yseg, axis=2, keepdims=True) + eps)
    yp = np.minimum(yseg * nc, xseg * (1 + 10 ** (-S.BETA / 20)))
    yp = yp - yp.mean(2, keepdims=True)
    xc = xseg - xseg.mean(2, keepdims=True)
    yp /= np.linalg.norm(yp, axis=2, keepdims=True) + eps
    xc /= np.linalg.norm(xc, axis=2, keepdims=True) + eps
    return np.sum(yp * xc) / (xc.shape[0] * xc.shape[1])


def _speechlike(n, fs, g, silence=True):
    t = torch.arange(n, dtype=torch.float64) / fs
    env = (torch.sin(2 * math.pi * 3 * t) ** 2) if silence else 1.0
    sig = env * (torch.sin(2 * math.pi * 220 * t) + 0.5 * torch.sin(2 * math.pi * 1330 * t)
                 + 0.3 * torch.randn(n, generator=g, dtype=torch.float64))
    if silence:
        sig[: n // 5] *= 1e-4  # a silent lead-in the frame removal must drop
    return sig


@pytest.mark.parametrize("fs", [8000, 10000, 16000])
def test_resample_matches_scipy(fs):
    import scipy.signal

    from torchmetrics_amd.functional.audio import stoi as S

    g = torch.Generator().manual_seed(fs)
    x = torch.randn(3, 4321, generator=g, dtype=torch.float64)
    h, up, down = S._octave_resample_filter(S.FS, fs)
    got = S._resample_poly(x, up, down, h)
    ref = np.stack([scipy.signal.resample_poly(r.numpy(), up, down, window=h) for r in x])
    np.testing.assert_allclose(got.numpy(), ref, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("fs", [8000, 16000])
@pytest.mark.parametrize("extended", [False, True])
def test_stoi_matches_numpy_transcription(fs, extended):
    g = torch.Generator().manual_seed(fs + extended)
    clean = torch.stack([_speechlike(fs * 2, fs, g), _speechlike(fs * 2, fs, g, silence=False)])
    noisy = clean + 0.8 * torch.randn(clean.shape, generator=g, dtype=torch.float64)
    got = short_time_objective_intelligibility(noisy, clean, fs, extended)
    ref = torch.tensor([_np_stoi(c.numpy(), n.numpy(), fs, extended) for c, n in zip(clean, noisy)])
    torch.testing.assert_close(got, ref, rtol=1e-9, atol=1e-9)
    # sanity: a clean signal scores (near) 1 and noise lowers it
    same = short_time_objective_intelligibility(clean, clean, fs, extended)
    assert torch.all(same > 0.99) and torch.all(got < same)


def test_stoi_module_and_short_input_warning():
    g = torch.Generator().manual_seed(0)
    clean = _speechlike(16000, 16000, g, silence=False).float()
    m = ShortTimeObjectiveIntelligibility(16000)
    m.update(clean[None] + 0.1 * torch.randn(1, 16000, generator=g), clean[None])
    assert 0 < float(m.compute()) < 1
    with pytest.warns(RuntimeWarning, match="Not enough STFT frames"):
        v = short_time_objective_intelligibility(torch.rand(2, 800), torch.rand(2, 800), 8000)
    assert torch.allclose(v, torch.full((2,), 1e-5, dtype=torch.float64))


@pytest.mark.gpu
def test_stoi_gpu_matches_cpu():
    g = torch.Generator().manual_seed(1)
    clean = torch.stack([_speechlike(32000, 16000, g) for _ in range(3)])
    noisy = clean + 0.5 * torch.randn(clean.shape, generator=g, dtype=torch.float64)
    for ext in (False, True):
        a = short_time_objective_intelligibility(noisy.cuda(), clean.cuda(), 16000, ext)
        b = short_time_objective_intelligibility(noisy, clean, 16000, ext)
        torch.testing.assert_close(a, b, rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_levinson_kernel_gpu():
    g = torch.Generator().manual_seed(5)
    for n_sys, L in ((1, 4), (37, 512), (5, 1500)):
        sig = torch.randn(n_sys, 4 * L, generator=g, dtype=torch.float64)
        r = torch.stack([torch.tensor(np.correlate(s.numpy(), s.numpy(), "full")[4 * L - 1:4 * L - 1 + L]) for s in sig])
        r[:, 0] += 1e-3
        b = torch.randn(n_sys, L, generator=g, dtype=torch.float64)
        x = ops.toeplitz_solve(r.cuda(), b.cuda()).cpu()
        ref = ops.toeplitz_solve(r, b)
        assert torch.allclose(x, ref, rtol=1e-6, atol=1e-8), (n_sys, L)
    # autograd through the kernel vs dense solve
    r = r[:2, :64].clone()
    b = b[:2, :64].clone()
    rc, bc = r.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    (ops.toeplitz_solve(rc, bc) ** 2).sum().backward()
    rr, bb = r.clone().requires_grad_(True), b.clone().requires_grad_(True)
    (ops.toeplitz_solve(rr, bb) ** 2).sum().backward()
    assert torch.allclose(rc.grad.cpu(), rr.grad, rtol=1e-6, atol=1e-8)
    assert torch.allclose(bc.grad.cpu(), bb.grad, rtol=1e-6, atol=1e-8)


@pytest.mark.gpu
def test_audio_modules_gpu():
    torch.manual_seed(1)
    p, t = torch.randn(8000), torch.randn(8000)
    assert torch.isclose(signal_distortion_ratio(p.cuda(), t.cuda()).cpu(), torch.tensor(-12.0589), atol=1e-3)
    for cls, fn, kw in (
        (SignalDistortionRatio, signal_distortion_ratio, {"filter_length": 32}),
        (ScaleInvariantSignalDistortionRatio, scale_invariant_signal_distortion_ratio, {}),
    ):
        test_modules_mean_of_batches(cls, fn, kw, device="cuda")


def test_srmr_docstring_and_module():
    from torchmetrics_amd.audio import SpeechReverberationModulationEnergyRatio
    from torchmetrics_amd.functional.audio import speech_reverberation_modulation_energy_ratio as srmr

    torch.manual_seed(1)
    preds = torch.randn(8000)
    out = srmr(preds, 8000)
    assert out.shape == (1,) and torch.isclose(out, torch.tensor([0.3354], dtype=torch.float64), atol=1e-4).all()
    m = SpeechReverberationModulationEnergyRatio(8000)
    m.update(preds)
    m.update(preds[None].repeat(2, 1))
    assert torch.isclose(m.compute(), torch.tensor(0.3354), atol=1e-4)
    assert srmr(torch.randn(2, 3, 4000), 8000, norm=True).shape == (2, 3)
    with pytest.raises(ModuleNotFoundError):
        srmr(preds, 8000, fast=True)  # FFT gammatonegram needs the `gammatone` package


def test_gammatone_design_unit_gain_at_centre():
    import numpy as np

    from torchmetrics_amd.functional.audio.srmr import _centre_freqs, _gammatone_sections, _make_erb_filters

    fs = 16000
    fc = _make_erb_filters(fs, 23, 125.0)
    imp = torch.zeros(1, 16384, dtype=torch.float64)
    imp[0, 0] = 1
    y = ops.biquad_cascade(imp, torch.from_numpy(_gammatone_sections(fc)), rep=23, clamp=False)
    y = y / torch.from_numpy(fc[:, 9]).reshape(-1, 1)
    spec = np.abs(np.fft.rfft(y.numpy(), axis=1))
    freqs = np.fft.rfftfreq(16384, 1 / fs)
    for i, c in enumerate(_centre_freqs(fs, 23, 125.0)):
        assert abs(spec[i, np.argmin(np.abs(freqs - c))] - 1.0) < 2e-2


@pytest.mark.gpu
def test_biquad_cascade_kernel_gpu():
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 2000, generator=g, dtype=torch.float64) * 0.1
    from torchmetrics_amd.functional.audio.srmr import _gammatone_sections, _make_erb_filters

    sec = torch.from_numpy(_gammatone_sections(_make_erb_filters(8000, 23, 125.0))) * 50
    for clamp in (False, True):
        got = ops.biquad_cascade(x.cuda(), sec, rep=23, clamp=clamp).cpu()
        ref = ops.biquad_cascade(x, sec, rep=23, clamp=clamp)
        assert torch.allclose(got, ref, rtol=1e-9, atol=1e-12)
    torch.manual_seed(1)
    preds = torch.randn(8000)
    from torchmetrics_amd.functional.audio import speech_reverberation_modulation_energy_ratio as srmr

    assert torch.isclose(srmr(preds.cuda(), 8000).cpu(), torch.tensor([0.3354], dtype=torch.float64), atol=1e-4).all()


@pytest.mark.gpu
def test_stoi_segment_kernel_ragged_batch(monkeypatch):
    """The segment kernel (csrc/audio/stoi.hip) on a batch whose signals keep different frame counts (silences), in
    fp32 and fp64, against the host path; the kernel is the one that runs."""
    calls = []
    real = ops.stoi_segments
    monkeypatch.setattr(ops, "stoi_segments", lambda *a: calls.append(1) or real(*a))
    g = torch.Generator().manual_seed(7)
    clean = torch.stack([_speechlike(48000, 16000, g), _speechlike(48000, 16000, g, silence=False),
                         _speechlike(48000, 16000, g)])
    clean[0, 20000:40000] = 0.0  # a long silence: fewer kept frames than the others
    noisy = clean + 0.4 * torch.randn(clean.shape, generator=g, dtype=torch.float64)
    for dt, tol in ((torch.float64, 1e-9), (torch.float32, 2e-5)):
        for ext in (False, True):
            a = short_time_objective_intelligibility(noisy.to(dt).cuda(), clean.to(dt).cuda(), 16000, ext)
            b = short_time_objective_intelligibility(noisy.to(dt), clean.to(dt), 16000, ext)
            torch.testing.assert_close(a.cpu(), b, rtol=tol, atol=tol)
    assert len(calls) == 4
