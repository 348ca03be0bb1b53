"""FID / KID / IS / MiFID against numpy/scipy oracles and the fp64-MFMA SYRK kernel against an fp64 GEMM."""
import numpy as np
import pytest
import torch
from scipy import linalg

from torchmetrics_amd import ops
from torchmetrics_amd.image import (
    FrechetInceptionDistance,
    InceptionScore,
    KernelInceptionDistance,
    MemorizationInformedFrechetInceptionDistance,
)
from torchmetrics_amd.models import InceptionV3Features
from tests.helpers import assert_close

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


class _Id(torch.nn.Module):
    def __init__(self, d):
        super().__init__()
        self.num_features = d

    def forward(self, x):
        return x


def _np_fid(r, f):
    r, f = r.double().cpu().numpy(), f.double().cpu().numpy()
    mu1, mu2 = r.mean(0), f.mean(0)
    s1, s2 = np.cov(r.T), np.cov(f.T)
    return ((mu1 - mu2) ** 2).sum() + np.trace(s1) + np.trace(s2) - 2 * np.trace(linalg.sqrtm(s1 @ s2).real)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("d", [16, 130])
def test_fid_matches_scipy(device, d):
    g = torch.Generator().manual_seed(0)
    real = torch.randn(300, d, generator=g)
    fake = torch.randn(300, d, generator=g) * 1.2 + 0.1
    m = FrechetInceptionDistance(feature=_Id(d)).to(device)
    for chunk in real.split(100):
        m.update(chunk.to(device), real=True)
    for chunk in fake.split(77):
        m.update(chunk.to(device), real=False)
    assert_close(m.compute(), _np_fid(real, fake), atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("case", ["random", "decay1e4", "decay1e10", "rank_deficient"])
def test_trace_sqrt_newton_schulz_matches_eigensolve(device, case):
    """The GEMM-only Newton-Schulz ``tr sqrt(Σ1 Σ2)`` (ROCm compute path) vs an fp64 eigensolve, including
    ill-conditioned and singular covariances (the unscaled tail must keep iterating until the trace settles)."""
    from torchmetrics_amd.image.generative import _trace_sqrt_newton_schulz, _trace_sqrt_product

    g = torch.Generator().manual_seed(1)
    d = 160
    n = 100 if case == "rank_deficient" else 2000
    decay = {"random": 0.0, "decay1e4": 4.0, "decay1e10": 10.0, "rank_deficient": 0.0}[case]
    sc = torch.logspace(0, -decay / 2, d, dtype=torch.float64)
    f1 = torch.randn(n, d, dtype=torch.float64, generator=g) * sc
    f2 = (torch.randn(n, d, dtype=torch.float64, generator=g) * 1.1 + 0.05) * sc
    s1, s2 = torch.cov(f1.T), torch.cov(f2.T)
    exact = torch.linalg.eigvals(s1 @ s2).real.clamp(min=0).sqrt().sum()
    got = _trace_sqrt_newton_schulz(s1.to(device), s2.to(device))
    if got is None:  # eigenvalues below the 1e-6 floor: the iteration declines and FID takes the eigensolve
        assert case in ("rank_deficient", "decay1e10")
        got = _trace_sqrt_product(s1.to(device), s2.to(device))
    # near-singular products limit the accuracy of the eigvals oracle itself to ~1e-8
    assert abs(float((got.cpu() - exact) / exact)) < (1e-7 if case in ("rank_deficient", "decay1e10") else 1e-9)


def test_fid_reset_real_features():
    m = FrechetInceptionDistance(feature=_Id(8), reset_real_features=False)
    m.update(torch.randn(10, 8), real=True)
    m.update(torch.randn(10, 8), real=False)
    m.reset()
    assert m.real_features_num_samples == 10 and m.fake_features_num_samples == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,dtype", [(1, 64, torch.float32), (1000, 2048, torch.float32), (517, 300, torch.bfloat16),
                                       (33, 129, torch.float16), (4096, 256, torch.float64)])
def test_syrk_kernel_vs_fp64_gemm(n, d, dtype):
    x = torch.randn(n, d, device="cuda").to(dtype)
    s0 = torch.randn(d, device="cuda", dtype=torch.float64)
    c0 = torch.randn(d, d, device="cuda", dtype=torch.float64)
    s, c = s0.clone(), c0.clone()
    ops.feature_moments_update(x, s, c)
    xd = x.double()
    torch.testing.assert_close(s, s0 + xd.sum(0), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(c, c0 + xd.t() @ xd, rtol=1e-12, atol=1e-9)


def _fid_states(m):
    names = ("real_features_sum", "real_features_cov_sum", "real_features_num_samples", "fake_features_sum",
             "fake_features_cov_sum", "fake_features_num_samples")
    return {k: getattr(m, k).clone() for k in names}


def _assert_states_close(a, b):
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=1e-11, atol=1e-8, msg=k)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("cap", [None, 1000])
def test_fid_staged_update_exact_state_semantics(device, cap):
    """Staged (deferred) SYRK: every observer of the states sees the eager values."""
    d = 96
    g = torch.Generator().manual_seed(3)
    batches = [(torch.randn(300, d, generator=g, dtype=torch.float64) * (1 + i % 3)).to(device) for i in range(9)]
    eager = FrechetInceptionDistance(feature=_Id(d)).to(device)
    eager._STAGE_MAX_ROWS = 0  # never stage
    staged = FrechetInceptionDistance(feature=_Id(d)).to(device)
    staged._STAGE_ON_CPU = True
    if cap is not None:
        staged._STAGE_MAX_ROWS = cap  # forces flushes between updates
    for i, b in enumerate(batches):
        for m in (eager, staged):
            m.update(b, real=i % 2 == 0)
    assert "_fid_hidden" in staged.__dict__ and staged.__dict__["_fid_hidden"]
    # attribute reads, state_dict and compute all see the eager values
    _assert_states_close(_fid_states(staged), _fid_states(eager))
    for m in (eager, staged):
        m.update(batches[0] * 0.5, real=False)
        m.persistent(True)
    sd_e, sd_s = eager.state_dict(), staged.state_dict()
    assert sd_e.keys() == sd_s.keys() and "real_features_cov_sum" in sd_e
    for k in sd_e:
        if k.endswith(("_sum", "_num_samples")):
            torch.testing.assert_close(sd_s[k], sd_e[k], rtol=1e-11, atol=1e-8)
    torch.testing.assert_close(staged.compute(), eager.compute(), rtol=1e-9, atol=1e-9)
    # reset drops staged rows; load_state_dict replaces them
    staged.update(batches[1], real=True)
    staged.reset()
    fresh = FrechetInceptionDistance(feature=_Id(d)).to(device)
    _assert_states_close(_fid_states(staged), _fid_states(fresh))
    staged.update(batches[2], real=True)
    staged.load_state_dict(sd_e)
    _assert_states_close(_fid_states(staged), {k: v for k, v in sd_e.items() if k in _fid_states(staged)})
    # clone with staged rows is independent and exact
    staged.update(batches[3], real=True)
    twin = staged.clone()
    eager.load_state_dict(sd_e)
    eager.update(batches[3], real=True)
    _assert_states_close(_fid_states(twin), _fid_states(eager))
    _assert_states_close(_fid_states(staged), _fid_states(eager))


@pytest.mark.gpu
def test_fid_staged_keep_real_features():
    d = 32
    g = torch.Generator().manual_seed(5)
    real, fake = torch.randn(200, d, generator=g).cuda(), torch.randn(200, d, generator=g).cuda()
    m = FrechetInceptionDistance(feature=_Id(d), reset_real_features=False).cuda()
    ref = FrechetInceptionDistance(feature=_Id(d)).cuda()
    ref._STAGE_MAX_ROWS = 0
    m.update(real, real=True)
    m.update(fake, real=False)
    m.reset()
    ref.update(real, real=True)
    _assert_states_close(_fid_states(m), _fid_states(ref))


def test_kid_matches_loop_oracle():
    g = torch.Generator().manual_seed(1)
    real, fake = torch.randn(120, 8, generator=g), torch.randn(120, 8, generator=g) + 0.3
    m = KernelInceptionDistance(feature=_Id(8), subsets=6, subset_size=40)
    m.update(real, True)
    m.update(fake, False)
    torch.manual_seed(7)
    mean, std = m.compute()
    torch.manual_seed(7)
    scores = []
    for _ in range(6):
        fr = real[torch.randperm(120)[:40]].double()
        ff = fake[torch.randperm(120)[:40]].double()
        k = lambda a, b: (a @ b.T / 8 + 1) ** 3  # noqa: E731
        kxx, kyy, kxy = k(fr, fr), k(ff, ff), k(fr, ff)
        mm = 40
        v = (kxx.sum() - kxx.diag().sum() + kyy.sum() - kyy.diag().sum()) / (mm * (mm - 1)) - 2 * kxy.sum() / mm**2
        scores.append(v)
    s = torch.stack(scores)
    assert_close(mean, s.mean(), atol=1e-5)
    assert_close(std, s.std(unbiased=False), atol=1e-5)


def test_inception_score_and_mifid():
    g = torch.Generator().manual_seed(2)
    logits = torch.randn(100, 10, generator=g)
    m = InceptionScore(feature=_Id(10), splits=1)
    m.update(logits)
    mean, _ = m.compute()
    p = logits.softmax(1)
    ref = (p * (p.log() - p.mean(0, keepdim=True).log())).sum(1).mean().exp()
    assert_close(mean, ref, atol=1e-5)
    mf = MemorizationInformedFrechetInceptionDistance(feature=_Id(6))
    real, fake = torch.randn(50, 6, generator=g), torch.randn(50, 6, generator=g)
    mf.update(real, True)
    mf.update(fake, False)
    assert torch.isfinite(mf.compute())


def test_inception_network_shapes():
    net = InceptionV3Features(["64", "2048", "logits_unbiased"])
    imgs = torch.randint(0, 255, (2, 3, 80, 80), dtype=torch.uint8)
    f64, f2048, logits = net(imgs)
    assert f64.shape == (2, 64) and f2048.shape == (2, 2048) and logits.shape == (2, 1008)
    fid = FrechetInceptionDistance(feature=64)
    fid.update(imgs, real=True)
    fid.update(imgs, real=False)
    assert fid.real_features_cov_sum.shape == (64, 64)


@pytest.mark.parametrize("device", DEVICES)
def test_fid_assigning_one_staged_state_keeps_sibling_rows(device):
    """Replacing one staged state (partial load) runs the staged rows into both first: the sibling keeps them."""
    d = 48
    g = torch.Generator().manual_seed(5)
    x = torch.randn(200, d, generator=g, dtype=torch.float64).to(device)
    eager = FrechetInceptionDistance(feature=_Id(d)).to(device)
    eager._STAGE_MAX_ROWS = 0
    staged = FrechetInceptionDistance(feature=_Id(d)).to(device)
    staged._STAGE_ON_CPU = True
    for m in (eager, staged):
        m.update(x, real=True)
    assert staged.__dict__.get("_fid_hidden")
    new_sum = torch.zeros(d, dtype=torch.float64, device=device)
    staged.real_features_sum = new_sum
    eager.real_features_sum = new_sum.clone()
    _assert_states_close(_fid_states(staged), _fid_states(eager))


@pytest.mark.gpu
def test_kid_gpu_full_subsets_is_exact_mmd():
    """Device-side draws: with subset_size == n every subset is a permutation of all rows, so the MMD is exact."""
    g = torch.Generator().manual_seed(11)
    real, fake = torch.randn(300, 64, generator=g), torch.randn(250, 64, generator=g) + 0.2
    m = KernelInceptionDistance(feature=_Id(64), subsets=4, subset_size=250).cuda()
    m.update(real[:250].cuda(), True)
    m.update(fake.cuda(), False)
    mean, std = m.compute()
    fr, ff = real[:250].double(), fake.double()
    k = lambda a, b: (a @ b.T / 64 + 1) ** 3  # noqa: E731
    kxx, kyy, kxy = k(fr, fr), k(ff, ff), k(fr, ff)
    v = (kxx.sum() - kxx.diag().sum() + kyy.sum() - kyy.diag().sum()) / (250 * 249) - 2 * kxy.sum() / 250**2
    assert_close(mean.cpu().double(), v, atol=1e-4, rtol=1e-4)
    assert float(std) < 1e-4


@pytest.mark.gpu
def test_mifid_cosine_distance_gpu_matches_cpu():
    from torchmetrics_amd.image.generative import _compute_cosine_distance

    g = torch.Generator().manual_seed(12)
    a, b = torch.randn(700, 64, generator=g), torch.randn(300, 64, generator=g)
    b[:50] = a[:50] * 2.0  # memorised rows: distance 0
    for eps in (0.1, 10.0):
        assert_close(_compute_cosine_distance(a.cuda(), b.cuda(), eps).cpu(), _compute_cosine_distance(a, b, eps),
                     atol=1e-5, rtol=1e-5)
