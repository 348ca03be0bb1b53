"""MFMA NT-GEMM epilogues (``csrc/pairwise/gemm_nt.hip``) vs fp64 PyTorch references of the same ops."""
import pytest
import torch

import torchmetrics_amd.functional as F
from torchmetrics_amd import ops

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
SHAPES = [(1, 1, 4), (37, 129, 20), (128, 128, 32), (300, 257, 100), (513, 64, 516)]


def _xy(n, m, d, seed=0, dev="cpu"):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, d, generator=g).to(dev), torch.randn(m, d, generator=g).to(dev) * 0.5 + 0.1


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n,m,d", SHAPES)
def test_store_asymmetric(device, n, m, d):
    x, y = _xy(n, m, d, dev=device)
    out = ops.gemm_nt(x, y, ops.GEMM_STORE, scale=0.5).cpu().double()
    ref = 0.5 * (x.double() @ y.double().T).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4 * d ** 0.5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n,m,d", SHAPES)
def test_euclid_vs_fp64_formula(device, n, m, d):
    x, y = _xy(n, m, d, seed=1, dev=device)
    y[: min(n, m) // 2] = x[: min(n, m) // 2] + 1e-4  # near duplicates: the cancellation guard must kick in
    nx, ny = (x * x).sum(1), (y * y).sum(1)
    out = ops.gemm_nt(x, y, ops.GEMM_EUCLID, nx, ny).cpu().double()
    ref = torch.cdist(x.double().cpu(), y.double().cpu())
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_poly_sum_and_row_reductions(device):
    x, y = _xy(300, 200, 64, seed=2, dev=device)
    k = ((x.double() @ y.double().T) / 64 + 1) ** 3
    part = ops.gemm_nt(x, y, ops.GEMM_POLY_SUM, scale=1 / 64, coef=1.0, degree=3)
    torch.testing.assert_close(part.sum().cpu(), k.sum().cpu(), rtol=1e-5, atol=1e-3)
    xx = ops.gemm_nt(x, x, ops.GEMM_POLY_SUM, scale=1 / 64, coef=1.0, degree=3, zero_diagonal=True)
    kxx = ((x.double() @ x.double().T) / 64 + 1) ** 3
    torch.testing.assert_close(xx.sum().cpu(), (kxx.sum() - kxx.diagonal().sum()).cpu(), rtol=1e-5, atol=1e-3)
    ix, iy = 1 / x.norm(dim=1), 1 / y.norm(dim=1)
    rmin = ops.gemm_nt(x, y, ops.GEMM_ROW_MIN, ix, iy).amin(-1).cpu()
    cos = (x.double() / x.double().norm(dim=1, keepdim=True)) @ (y.double() / y.double().norm(dim=1, keepdim=True)).T
    torch.testing.assert_close(rmin.double(), (1 - cos.abs()).amin(1).cpu(), rtol=1e-5, atol=1e-6)
    rsum = ops.gemm_nt(x, y, ops.GEMM_ROW_SUM, scale=2.0).sum(-1).cpu()
    torch.testing.assert_close(rsum.double(), 2 * (x.double() @ y.double().T).sum(1).cpu(), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("device", DEVICES)
def test_batched_store(device):
    g = torch.Generator().manual_seed(3)
    x, y = torch.randn(3, 70, 36, generator=g).to(device), torch.randn(3, 50, 36, generator=g).to(device)
    out = ops.gemm_nt(x, y, ops.GEMM_STORE).cpu().double()
    torch.testing.assert_close(out, torch.bmm(x.double(), y.double().transpose(1, 2)).cpu(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("zd", [False, True])
def test_pairwise_functionals_route_to_mfma(zd):
    x, y = _xy(1000, 700, 128, seed=4, dev="cuda")
    for fn, ref in [
        (F.pairwise_euclidean_distance, lambda a, b: torch.cdist(a, b)),
        (F.pairwise_linear_similarity, lambda a, b: a @ b.T),
        (F.pairwise_cosine_similarity,
         lambda a, b: (a / a.norm(dim=1, keepdim=True)) @ (b / b.norm(dim=1, keepdim=True)).T),
    ]:
        out = fn(x, x, zero_diagonal=zd).double().cpu()
        r = ref(x.double().cpu(), x.double().cpu())
        if zd:
            r.fill_diagonal_(0)
        torch.testing.assert_close(out, r, rtol=1e-5, atol=1e-4)
        out = fn(x, y).double().cpu()
        torch.testing.assert_close(out, ref(x.double().cpu(), y.double().cpu()), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
def test_gathered_batched_poly_sum(device):
    """KID path: per-subset row gathers inside the GEMM == explicit gathers + poly kernel sums."""
    g = torch.Generator().manual_seed(5)
    real, fake = torch.randn(500, 64, generator=g).to(device), torch.randn(400, 64, generator=g).to(device)
    ir = torch.stack([torch.randperm(500, generator=g)[:130] for _ in range(3)]).to(device)
    jf = torch.stack([torch.randperm(400, generator=g)[:130] for _ in range(3)]).to(device)
    out = ops.gemm_nt(real, fake, ops.GEMM_POLY_SUM, scale=1 / 64, coef=1.0, degree=3, idx_x=ir, idx_y=jf)
    fr, ff = real[ir].double(), fake[jf].double()
    ref = ((torch.bmm(fr, ff.transpose(1, 2)) / 64 + 1) ** 3).sum((1, 2))
    torch.testing.assert_close(out.sum(-1).cpu(), ref.cpu(), rtol=1e-5, atol=1e-3)
    same = ops.gemm_nt(real, real, ops.GEMM_POLY_SUM, scale=1 / 64, coef=1.0, degree=3, idx_x=ir, idx_y=ir,
                       zero_diagonal=True)
    k = (torch.bmm(fr, fr.transpose(1, 2)) / 64 + 1) ** 3
    ref = k.sum((1, 2)) - k.diagonal(dim1=1, dim2=2).sum(-1)
    torch.testing.assert_close(same.sum(-1).cpu(), ref.cpu(), rtol=1e-5, atol=1e-3)
