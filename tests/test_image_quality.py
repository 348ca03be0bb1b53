"""Image quality metrics vs independent numpy / scipy oracles (reference test model: ``T/image``).

SSIM / UQI oracles evaluate every valid window explicitly with ``sliding_window_view`` (no convolution); the GPU
cases exercise the fused HIP window kernel.
"""
import math

import numpy as np
import pytest
import torch
from numpy.lib.stride_tricks import sliding_window_view
from scipy import signal

import torchmetrics_amd.functional as F
from torchmetrics_amd import image as I
from tests.helpers import assert_close, run_class_test

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _np(x):
    return x.detach().cpu().double().numpy()


def _gauss(k, s):
    x = np.arange(k) - (k - 1) / 2
    g = np.exp(-0.5 * (x / s) ** 2)
    return g / g.sum()


def _window_moments(p, t, w2):
    """Weighted moments of every valid window of [H, W] planes with 2-D weights w2."""
    kh, kw = w2.shape
    wp, wt = sliding_window_view(p, (kh, kw)), sliding_window_view(t, (kh, kw))
    m = lambda a: (a * w2).sum((-1, -2))  # noqa: E731
    return m(wp), m(wt), m(wp * wp), m(wt * wt), m(wp * wt)


def _ssim_oracle(preds, target, sigma=1.5, data_range=None, k1=0.01, k2=0.03, gaussian=True, ks=11, cs=False):
    p, t = _np(preds), _np(target)
    dr = max(p.max() - p.min(), t.max() - t.min()) if data_range is None else data_range
    c1, c2 = (k1 * dr) ** 2, (k2 * dr) ** 2
    gk = int(3.5 * sigma + 0.5) * 2 + 1
    w = np.outer(_gauss(gk, sigma), _gauss(gk, sigma)) if gaussian else np.full((ks, ks), 1 / ks**2)
    out, out_cs = [], []
    for b in range(p.shape[0]):
        vals, css = [], []
        for c in range(p.shape[1]):
            mx, my, exx, eyy, exy = _window_moments(p[b, c], t[b, c], w)
            sxx, syy, sxy = np.maximum(exx - mx**2, 0), np.maximum(eyy - my**2, 0), exy - mx * my
            up, lo = 2 * sxy + c2, sxx + syy + c2
            vals.append(((2 * mx * my + c1) * up) / ((mx**2 + my**2 + c1) * lo))
            css.append(up / lo)
        out.append(np.mean(vals))
        out_cs.append(np.mean(css))
    return (np.array(out), np.array(out_cs)) if cs else np.array(out)


def _imgs(seed=0, b=4, c=3, h=48, w=40):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(2, b, c, h, w, generator=g)
    p = (t + 0.1 * torch.randn(2, b, c, h, w, generator=g)).clamp(0, 1)
    return p, t


# ------------------------------------------------------------------------------------------------------- SSIM
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("sigma", [1.5, 0.8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_ssim_vs_window_oracle(device, sigma, dtype):
    p, t = _imgs()
    p, t = p.to(dtype), t.to(dtype)
    run_class_test(p, t, I.StructuralSimilarityIndexMeasure, lambda a, b: _ssim_oracle(a, b, sigma).mean(),
                   {"sigma": sigma, "data_range": 1.0}, atol=2e-5, device=device)


@pytest.mark.parametrize("device", DEVICES)
def test_ssim_variants(device):
    p, t = _imgs(seed=1)
    p0, t0 = p[0].to(device), t[0].to(device)
    # data_range=None (device-side range), uniform window, contrast sensitivity, per-image reduction
    assert_close(F.structural_similarity_index_measure(p0, t0), _ssim_oracle(p[0], t[0]).mean(), atol=2e-5)
    assert_close(F.structural_similarity_index_measure(p0, t0, gaussian_kernel=False, kernel_size=11, data_range=1.0),
                 _ssim_oracle(p[0], t[0], data_range=1.0, gaussian=False).mean(), atol=2e-5)
    sim, cs = F.structural_similarity_index_measure(p0, t0, data_range=1.0, reduction="none",
                                                     return_contrast_sensitivity=True)
    osim, ocs = _ssim_oracle(p[0], t[0], data_range=1.0, cs=True)
    assert_close(sim, osim, atol=2e-5)
    assert_close(cs, ocs, atol=2e-5)
    val, full = F.structural_similarity_index_measure(p0, t0, data_range=1.0, return_full_image=True)
    assert full.shape == p0.shape
    assert_close(val, osim.mean(), atol=2e-5)
    # data_range tuple clamps
    assert_close(F.structural_similarity_index_measure(p0 * 2, t0 * 2, data_range=(0.0, 1.0)),
                 _ssim_oracle((p[0] * 2).clamp(0, 1), (t[0] * 2).clamp(0, 1), data_range=1.0).mean(), atol=2e-5)


def test_ssim_3d_and_grad():
    g = torch.Generator().manual_seed(2)
    t = torch.rand(2, 1, 16, 16, 16, generator=g)
    p = (t + 0.05 * torch.randn(2, 1, 16, 16, 16, generator=g)).clamp(0, 1)
    val = F.structural_similarity_index_measure(p, t, data_range=1.0, kernel_size=5, sigma=0.7)
    assert 0 < val < 1
    p2 = p[:, :, 0].clone().requires_grad_(True)
    F.structural_similarity_index_measure(p2, t[:, :, 0], data_range=1.0).backward()
    assert p2.grad is not None and torch.isfinite(p2.grad).all()


@pytest.mark.parametrize("device", DEVICES)
def test_ms_ssim(device):
    g = torch.Generator().manual_seed(3)
    t = torch.rand(2, 3, 1, 180, 180, generator=g)
    p = (t + 0.05 * torch.randn(t.shape, generator=g)).clamp(0, 1)
    betas = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)

    def oracle(pp, tt):
        pp, tt = pp.double(), tt.double()
        css = []
        for _ in range(len(betas)):
            s, c = _ssim_oracle(pp, tt, data_range=1.0, cs=True)
            css.append(np.maximum(c, 0))
            pp = torch.nn.functional.avg_pool2d(pp, 2)
            tt = torch.nn.functional.avg_pool2d(tt, 2)
        css[-1] = np.maximum(s, 0)
        return np.prod(np.stack(css) ** np.array(betas)[:, None], 0).mean()

    run_class_test(p, t, I.MultiScaleStructuralSimilarityIndexMeasure, oracle, {"data_range": 1.0}, atol=1e-5,
                   device=device)


# -------------------------------------------------------------------------------------------------------- UQI
def _uqi_oracle(preds, target, ks=11, sigma=1.5):
    p, t = _np(preds), _np(target)
    w = np.outer(_gauss(ks, sigma), _gauss(ks, sigma))
    eps = np.finfo(np.float32).eps
    vals = []
    for b in range(p.shape[0]):
        for c in range(p.shape[1]):
            mx, my, exx, eyy, exy = _window_moments(p[b, c], t[b, c], w)
            sxx, syy, sxy = np.maximum(exx - mx**2, 0), np.maximum(eyy - my**2, 0), exy - mx * my
            vals.append(((2 * mx * my) * 2 * sxy) / ((mx**2 + my**2) * (sxx + syy) + eps))
    return np.mean(vals)


@pytest.mark.parametrize("device", DEVICES)
def test_uqi(device):
    p, t = _imgs(seed=4)
    run_class_test(p, t, I.UniversalImageQualityIndex, _uqi_oracle, {}, atol=5e-5, device=device)
    none = F.universal_image_quality_index(p[0].to(device), t[0].to(device), reduction="none")
    assert none.shape == (4, 3, 38, 30)
    assert_close(none.mean(), _uqi_oracle(p[0], t[0]), atol=5e-5)


# --------------------------------------------------------------------------------------- simple pixel metrics
@pytest.mark.parametrize("device", DEVICES)
def test_psnr_family(device):
    p, t = _imgs(seed=5)
    def psnr(a, b):
        a, b = _np(a), _np(b)
        return 10 * np.log10((b.max() - b.min()) ** 2 / np.mean((a - b) ** 2))
    # data_range=None tracks min/max of the targets across updates; the oracle uses the same over all batches
    run_class_test(p, t, I.PeakSignalNoiseRatio, psnr, {}, atol=1e-4, device=device, check_batch=False)
    run_class_test(p, t, I.PeakSignalNoiseRatio, lambda a, b: 10 * np.log10(1 / np.mean((_np(a) - _np(b)) ** 2)),
                   {"data_range": 1.0}, atol=1e-4, device=device)
    per = F.peak_signal_noise_ratio(p[0].to(device), t[0].to(device), data_range=1.0, dim=(1, 2, 3), reduction="none")
    ref = 10 * np.log10(1 / ((_np(p[0]) - _np(t[0])) ** 2).mean((1, 2, 3)))
    assert_close(per, ref, atol=1e-4)


def _bef_oracle(x, bs=8):
    x = _np(x)[:, 0]
    _, h, w = x.shape
    hb = [j for j in range(w - 1) if j % bs == bs - 1]
    hbc = [j for j in range(w - 1) if j % bs != bs - 1]
    vb = [i for i in range(h - 1) if i % bs == bs - 1]
    vbc = [i for i in range(h - 1) if i % bs != bs - 1]
    d_b = sum(((x[:, :, j] - x[:, :, j + 1]) ** 2).sum() for j in hb) + sum(((x[:, i] - x[:, i + 1]) ** 2).sum()
                                                                            for i in vb)
    d_bc = sum(((x[:, :, j] - x[:, :, j + 1]) ** 2).sum() for j in hbc) + sum(((x[:, i] - x[:, i + 1]) ** 2).sum()
                                                                              for i in vbc)
    n_hb = h * (w / bs) - 1
    n_hbc = h * (w - 1) - n_hb
    n_vb = w * (h / bs) - 1
    n_vbc = w * (h - 1) - n_vb
    d_b /= n_hb + n_vb
    d_bc /= n_hbc + n_vbc
    t = math.log2(bs) / math.log2(min(h, w)) if d_b > d_bc else 0
    return t * (d_b - d_bc)


def test_psnrb():
    g = torch.Generator().manual_seed(6)
    t = torch.rand(2, 1, 32, 32, generator=g)
    p = t.clone()
    p[..., 7, :] += 0.3  # a blocking artefact on a block boundary
    mse = ((_np(p) - _np(t)) ** 2).mean() + _bef_oracle(p)
    assert_close(F.peak_signal_noise_ratio_with_blocked_effect(p, t), 10 * np.log10(1 / mse), atol=1e-4)
    m = I.PeakSignalNoiseRatioWithBlockedEffect()
    m.update(p, t)
    assert_close(m.compute(), 10 * np.log10(1 / mse), atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_sam_ergas_tv_gradients(device):
    p, t = _imgs(seed=7)
    p, t = p + 0.1, t + 0.1

    def sam(a, b):
        a, b = _np(a), _np(b)
        cos = (a * b).sum(1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))
        return np.arccos(np.clip(cos, -1, 1)).mean()

    def ergas(a, b, ratio=4):
        a, b = _np(a), _np(b)
        bb, c = a.shape[:2]
        rmse = np.sqrt(((a - b) ** 2).reshape(bb, c, -1).mean(-1))
        return (100 * ratio * np.sqrt(((rmse / b.reshape(bb, c, -1).mean(-1)) ** 2).sum(1) / c)).mean()

    run_class_test(p, t, I.SpectralAngleMapper, sam, {}, atol=1e-5, device=device)
    run_class_test(p, t, I.ErrorRelativeGlobalDimensionlessSynthesis, ergas, {}, atol=1e-3, device=device)
    img = p[0].to(device)
    tv = np.abs(np.diff(_np(img), axis=2)).sum() + np.abs(np.diff(_np(img), axis=3)).sum()
    assert_close(F.total_variation(img), tv, atol=1e-3)
    m = I.TotalVariation(reduction="mean").to(device)
    m.update(img)
    assert_close(m.compute(), tv / img.shape[0], atol=1e-3)
    dy, dx = F.image_gradients(img)
    assert_close(dy[..., :-1, :], np.diff(_np(img), axis=2), atol=1e-6)
    assert_close(dx[..., -1], np.zeros_like(_np(img)[..., -1]), atol=0)


def _box_sym(x, w):
    """Reference uniform filter: symmetric pad (w//2 before, w//2 + w%2 - 1 after), box mean over valid windows."""
    before, after = w // 2, w // 2 + w % 2 - 1
    xp = np.pad(x, ((0, 0), (0, 0), (before, after), (before, after)), mode="symmetric")
    return sliding_window_view(xp, (w, w), axis=(2, 3)).mean((-1, -2))


def test_rmse_sw_and_rase():
    p, t = _imgs(seed=8, h=24, w=24)
    p, t = p[0] + 0.2, t[0] + 0.2
    w = 8
    rmse_map = np.sqrt(_box_sym((_np(t) - _np(p)) ** 2, w))
    crop = round(w / 2)
    ref = rmse_map[:, :, crop:-crop, crop:-crop].sum(0).mean() / p.shape[0]
    assert_close(F.root_mean_squared_error_using_sliding_window(p, t, w), ref, atol=1e-5)
    m = I.RootMeanSquaredErrorUsingSlidingWindow(window_size=w)
    m.update(p, t)
    assert_close(m.compute(), ref, atol=1e-5)
    rmse_map_mean = rmse_map.sum(0) / p.shape[0]
    tmean = (_box_sym(_np(t), w) / w**2).sum(0) / p.shape[0]
    rase_map = 100 / tmean.mean(0) * np.sqrt((rmse_map_mean**2).mean(0))
    assert_close(F.relative_average_spectral_error(p, t, w), rase_map[crop:-crop, crop:-crop].mean(), atol=1e-3)


def test_scc_vs_scipy():
    p, t = _imgs(seed=9, h=32, w=32)
    p, t = p[0], t[0]
    hp = np.array([[-1, -1, -1], [-1, 8, -1], [-1, -1, -1]], dtype=np.float64)
    ws = 8
    vals = []
    for b in range(p.shape[0]):
        per_c = []
        for c in range(p.shape[1]):
            ph = signal.convolve2d(_np(p)[b, c], hp, mode="same", boundary="symm") * 2
            th = signal.convolve2d(_np(t)[b, c], hp, mode="same", boundary="symm") * 2
            lo, hi = math.ceil((ws - 1) / 2), (ws - 1) // 2
            box = lambda a: sliding_window_view(np.pad(a, ((lo, hi), (lo, hi))), (ws, ws)).mean((-1, -2))  # noqa
            mp, mt = box(ph), box(th)
            vp, vt = np.maximum(box(ph**2) - mp**2, 0), np.maximum(box(th**2) - mt**2, 0)
            cov = box(ph * th) - mp * mt
            den = np.sqrt(vt) * np.sqrt(vp)
            per_c.append(np.where(den == 0, 0, cov / np.where(den == 0, 1, den)))
        vals.append(np.mean(per_c))
    assert_close(F.spatial_correlation_coefficient(p, t), np.mean(vals), atol=1e-4)
    m = I.SpatialCorrelationCoefficient()
    m.update(p, t)
    assert_close(m.compute(), np.mean(vals), atol=1e-4)


def test_vif_vs_numpy():
    g = torch.Generator().manual_seed(10)
    t = torch.rand(2, 1, 64, 64, generator=g) * 255
    p = (t + 20 * torch.randn(t.shape, generator=g)).clamp(0, 255)
    sn, eps = 2.0, 1e-10

    def vif(ref, dist):
        num = den = 0.0
        for scale in range(4):
            n = 2.0 ** (4 - scale) + 1
            x = np.arange(n) - (n - 1) / 2
            win = np.exp(-(x[None] ** 2 + x[:, None] ** 2) / (2 * (n / 5) ** 2))
            win /= win.sum()
            if scale > 0:
                ref = signal.correlate2d(ref, win, mode="valid")[::2, ::2]
                dist = signal.correlate2d(dist, win, mode="valid")[::2, ::2]
            f = lambda a: signal.correlate2d(a, win, mode="valid")  # noqa: E731
            mu1, mu2 = f(ref), f(dist)
            s1, s2 = np.maximum(f(ref * ref) - mu1**2, 0), np.maximum(f(dist * dist) - mu2**2, 0)
            s12 = f(ref * dist) - mu1 * mu2
            gg = s12 / (s1 + eps)
            sv = s2 - gg * s12
            gg[s1 < eps] = 0
            sv[s1 < eps] = s2[s1 < eps]
            s1[s1 < eps] = 0
            gg[s2 < eps] = 0
            sv[s2 < eps] = 0
            sv[gg < 0] = s2[gg < 0]
            gg[gg < 0] = 0
            sv = np.maximum(sv, eps)
            num += np.log10(1 + gg**2 * s1 / (sv + sn)).sum()
            den += np.log10(1 + s1 / sn).sum()
        return num / den

    ref = np.mean([vif(_np(t)[b, 0], _np(p)[b, 0]) for b in range(2)])
    assert_close(F.visual_information_fidelity(p, t), ref, atol=1e-4)
    m = I.VisualInformationFidelity()
    m.update(p, t)
    assert_close(m.compute(), ref, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_pansharpening(device):
    g = torch.Generator().manual_seed(11)
    preds = torch.rand(2, 3, 32, 32, generator=g).to(device)
    ms = torch.rand(2, 3, 16, 16, generator=g).to(device)
    pan = torch.rand(2, 3, 32, 32, generator=g).to(device)
    pan_lr = torch.rand(2, 3, 16, 16, generator=g).to(device)

    def uqi_pair(a, b):
        return _uqi_oracle(a.unsqueeze(1), b.unsqueeze(1))

    def band_matrix(x):
        c = x.shape[1]
        m = np.zeros((c, c))
        for i in range(c):
            for j in range(i + 1, c):
                m[i, j] = m[j, i] = uqi_pair(x[:, i], x[:, j])
        return m

    d_lambda = np.abs(band_matrix(ms) - band_matrix(preds)).sum() / (3 * 2)
    assert_close(F.spectral_distortion_index(preds, ms), d_lambda, atol=1e-4)
    m1 = np.array([uqi_pair(ms[:, i], pan_lr[:, i]) for i in range(3)])
    m2 = np.array([uqi_pair(preds[:, i], pan[:, i]) for i in range(3)])
    d_s = np.abs(m1 - m2).mean()
    assert_close(F.spatial_distortion_index(preds, ms, pan, pan_lr), d_s, atol=1e-4)
    qnr = I.QualityWithNoReference().to(device)
    qnr.update(preds, {"ms": ms, "pan": pan, "pan_lr": pan_lr})
    assert_close(qnr.compute(), (1 - d_lambda) * (1 - d_s), atol=1e-4)
    # pan_lr derived from pan (box filter + bilinear resize) just has to run and be finite
    assert torch.isfinite(F.spatial_distortion_index(preds, ms, pan))
