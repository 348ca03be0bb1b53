"""Fused HIP kernels for the SNR family (csrc/audio/snr.hip), Inception Score (csrc/image/inception_score.hip) and
hinge loss (csrc/classification/hinge.hip) against fp64 evaluations of the reference formulas on the host."""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops
from torchmetrics_amd.functional import audio as FA

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _signals(shape, seed, noise=0.3):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g)
    p = 0.8 * t + noise * torch.randn(*shape, generator=g) + 0.1
    return p, t


@pytest.mark.parametrize("zero_mean", [False, True])
@pytest.mark.parametrize("noise", [0.3, 1e-3])  # 1e-3: ~60 dB, where E[x^2]-style shortcuts lose digits
def test_snr_and_si_sdr(zero_mean, noise):
    p, t = _signals((3, 2, 16000), 1, noise)
    for fn in (FA.signal_noise_ratio, FA.scale_invariant_signal_distortion_ratio):
        ref = fn(p.double(), t.double(), zero_mean=zero_mean)  # host ATen path, fp64
        got = fn(p.to(DEV), t.to(DEV), zero_mean=zero_mean)
        assert got.shape == ref.shape and got.dtype == torch.float32
        torch.testing.assert_close(got.cpu().double(), ref, atol=2e-3, rtol=1e-4)
    ref = FA.scale_invariant_signal_noise_ratio(p.double(), t.double())
    torch.testing.assert_close(FA.scale_invariant_signal_noise_ratio(p.to(DEV), t.to(DEV)).cpu().double(), ref,
                               atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("scale_invariant", [False, True])
@pytest.mark.parametrize("zero_mean", [False, True])
def test_sa_sdr(scale_invariant, zero_mean):
    p, t = _signals((4, 3, 8000), 2)
    ref = FA.source_aggregated_signal_distortion_ratio(p.double(), t.double(), scale_invariant, zero_mean)
    got = FA.source_aggregated_signal_distortion_ratio(p.to(DEV), t.to(DEV), scale_invariant, zero_mean)
    torch.testing.assert_close(got.cpu().double(), ref, atol=2e-3, rtol=1e-4)


def test_c_si_snr_and_grad_path():
    p, t = _signals((2, 65, 50, 2), 3)
    ref = FA.complex_scale_invariant_signal_noise_ratio(p.double(), t.double())
    got = FA.complex_scale_invariant_signal_noise_ratio(p.to(DEV), t.to(DEV))
    torch.testing.assert_close(got.cpu().double(), ref, atol=2e-3, rtol=1e-4)
    # differentiable path (ATen formula) still used when a gradient is needed
    pg = p[..., 0].to(DEV).requires_grad_()
    out = FA.scale_invariant_signal_distortion_ratio(pg, t[..., 0].to(DEV)).sum()
    out.backward()
    assert pg.grad is not None and torch.isfinite(pg.grad).all()


def _is_reference(logits, perm, splits):
    x = logits.double()[perm]
    prob, logp = x.softmax(1), x.log_softmax(1)
    kls = [(p * (lp - p.mean(0, keepdim=True).log())).sum(1).mean().exp()
           for p, lp in zip(prob.chunk(splits), logp.chunk(splits))]
    k = torch.stack(kls)
    return k.mean(), k.std()


@pytest.mark.parametrize("n,splits", [(1000, 10), (997, 7), (50, 6)])
def test_inception_score_kernel(n, splits):
    g = torch.Generator().manual_seed(n)
    logits = 3 * torch.randn(n, 1008, generator=g)
    perm = torch.randperm(n, generator=g)
    mean, std = _is_reference(logits, perm, splits)
    out = ops.inception_score(logits.to(DEV), perm, splits).cpu()
    torch.testing.assert_close(out[0].double(), mean, rtol=2e-5, atol=1e-5)
    torch.testing.assert_close(out[1].double(), std, rtol=2e-3, atol=1e-5)


def test_inception_score_module_matches_host():
    torch.manual_seed(0)
    feats = 2 * torch.randn(400, 1008)
    from torchmetrics_amd.image.generative import InceptionScore

    gpu = InceptionScore(feature=torch.nn.Identity(), splits=5).to(DEV)
    cpu = InceptionScore(feature=torch.nn.Identity(), splits=5)
    gpu.features.append(feats.to(DEV))
    cpu.features.append(feats.clone())
    gpu._update_count = cpu._update_count = 1
    torch.manual_seed(7)
    a = gpu.compute()
    torch.manual_seed(7)
    b = cpu.compute()
    torch.testing.assert_close(a[0].cpu(), b[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(a[1].cpu(), b[1], rtol=5e-3, atol=1e-5)


@pytest.mark.parametrize("squared", [False, True])
@pytest.mark.parametrize("probs", [False, True])
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_hinge_binary(squared, probs, ignore_index):
    g = torch.Generator().manual_seed(int(squared) + 2 * int(probs))
    preds = torch.rand(5000, generator=g) if probs else 3 * torch.randn(5000, generator=g)
    target = torch.randint(0, 2, (5000,), generator=g)
    if ignore_index is not None:
        target[::7] = ignore_index
    gpu = tm.BinaryHingeLoss(squared=squared, ignore_index=ignore_index).to(DEV)
    cpu = tm.BinaryHingeLoss(squared=squared, ignore_index=ignore_index)
    for i in range(3):
        sl = slice(i * 1500, (i + 1) * 1500 + 500)
        gpu.update(preds[sl].to(DEV), target[sl].to(DEV))
        cpu.update(preds[sl], target[sl])
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["crammer-singer", "one-vs-all"])
@pytest.mark.parametrize("squared", [False, True])
@pytest.mark.parametrize("probs", [False, True])
def test_hinge_multiclass(mode, squared, probs):
    g = torch.Generator().manual_seed(len(mode) + int(squared))
    c = 7
    preds = torch.randn(3000, c, generator=g)
    if probs:
        preds = preds.softmax(1)
    target = torch.randint(0, c, (3000,), generator=g)
    target[::11] = -100
    gpu = tm.MulticlassHingeLoss(c, squared=squared, multiclass_mode=mode, ignore_index=-100).to(DEV)
    cpu = tm.MulticlassHingeLoss(c, squared=squared, multiclass_mode=mode, ignore_index=-100)
    for sl in (slice(0, 1000), slice(1000, 3000)):
        gpu.update(preds[sl].to(DEV), target[sl].to(DEV))
        cpu.update(preds[sl], target[sl])
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)


def test_hinge_bad_target_raises_at_compute():
    m = tm.BinaryHingeLoss().to(DEV)
    m.update(torch.randn(10, device=DEV), torch.tensor([0, 1, 2, 0, 1, 0, 1, 0, 1, 0], device=DEV))
    with pytest.raises((RuntimeError, ValueError)):
        m.compute()
    m = tm.MulticlassHingeLoss(3).to(DEV)
    m.update(torch.randn(4, 3, device=DEV), torch.tensor([0, 1, 5, 2], device=DEV))
    with pytest.raises((RuntimeError, ValueError)):
        m.compute()


@pytest.mark.parametrize("n", [1, 2, 6, 9, 40, 70])
@pytest.mark.parametrize("maximize", [False, True])
def test_linear_sum_assignment_matches_scipy(n, maximize):
    from scipy.optimize import linear_sum_assignment

    g = torch.Generator().manual_seed(n)
    cost = torch.randn(12, n, n, generator=g, dtype=torch.float64)
    got = ops.linear_sum_assignment(cost.to(DEV), maximize).cpu()
    for b in range(12):
        r, c = linear_sum_assignment(cost[b].numpy(), maximize)
        best = cost[b][r, c].sum()
        mine = cost[b][torch.arange(n), got[b]].sum()
        assert sorted(got[b].tolist()) == list(range(n))  # a permutation
        torch.testing.assert_close(mine, best, rtol=1e-12, atol=1e-9)


def test_pit_many_speakers_on_device():
    from torchmetrics_amd.functional.audio import permutation_invariant_training, scale_invariant_signal_distortion_ratio

    g = torch.Generator().manual_seed(0)
    t = torch.randn(3, 7, 400, generator=g)
    perm = torch.stack([torch.randperm(7, generator=g) for _ in range(3)])
    p = torch.gather(t, 1, perm[:, :, None].expand(-1, -1, 400)) + 0.05 * torch.randn(3, 7, 400, generator=g)
    best_cpu, perm_cpu = permutation_invariant_training(p, t, scale_invariant_signal_distortion_ratio, "speaker-wise",
                                                        "max")
    best, pm = permutation_invariant_training(p.to(DEV), t.to(DEV), scale_invariant_signal_distortion_ratio,
                                              "speaker-wise", "max")
    assert torch.equal(pm.cpu(), perm_cpu)
    torch.testing.assert_close(best.cpu(), best_cpu, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("shape", [(2, 1, 41, 41), (3, 3, 64, 70), (1, 2, 130, 97)])
def test_vif_fused_scales_match_torch_path(shape, dtype):
    from torchmetrics_amd.functional.image import spatial as S

    g = torch.Generator().manual_seed(shape[-1])
    t = torch.rand(*shape, generator=g, dtype=torch.float64).to(dtype)
    p = (t + 0.1 * torch.randn(*shape, generator=g, dtype=torch.float64).to(dtype)).clamp(0, 1)
    got = S.visual_information_fidelity(p.cuda(), t.cuda()).cpu()
    want = S.visual_information_fidelity(p, t)
    torch.testing.assert_close(got, want, atol=1e-5 if dtype == torch.float32 else 1e-10, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("window_size", [3, 8, 11])
@pytest.mark.parametrize("reduction", ["mean", "none"])
def test_scc_fused_matches_torch_path(window_size, reduction):
    from torchmetrics_amd.functional.image import spatial_correlation_coefficient

    g = torch.Generator().manual_seed(window_size)
    p = torch.rand(3, 2, 50, 45, generator=g)
    t = (p + 0.2 * torch.rand(3, 2, 50, 45, generator=g)).clamp(0, 1)
    got = spatial_correlation_coefficient(p.cuda(), t.cuda(), window_size=window_size, reduction=reduction).cpu()
    want = spatial_correlation_coefficient(p, t, window_size=window_size, reduction=reduction)
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-4)
    m_gpu = tm.image.SpatialCorrelationCoefficient(window_size=window_size).cuda()
    m_cpu = tm.image.SpatialCorrelationCoefficient(window_size=window_size)
    m_gpu.update(p.cuda(), t.cuda())
    m_cpu.update(p, t)
    torch.testing.assert_close(m_gpu.compute().cpu(), m_cpu.compute(), atol=1e-5, rtol=1e-4)
