"""The 256 x 256-tile MFMA NT-GEMM (``gemm_nt_big_kernel``, global_load_lds staging) on shapes that select it: every
epilogue against an fp64 PyTorch reference, partial tiles on both sides, batched and row-gathered operands."""
import pytest
import torch

from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _xy(n, m, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, d, generator=g), torch.randn(m, d, generator=g) * 0.5 + 0.1


@pytest.mark.parametrize("n,m,d", [(4096, 4096, 64), (4100, 4097, 96), (2304, 8200, 256)])
def test_big_store(n, m, d):
    x, y = _xy(n, m, d)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_STORE, scale=0.5).cpu().double()
    ref = 0.5 * (x.double() @ y.double().T)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4 * d ** 0.5)


def test_big_euclid_cosine():
    n, m, d = 4100, 4097, 96
    x, y = _xy(n, m, d, 1)
    y[:1000] = x[:1000] + 1e-4
    nx, ny = (x * x).sum(1), (y * y).sum(1)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_EUCLID, nx.to(DEV), ny.to(DEV)).cpu().double()
    torch.testing.assert_close(out, torch.cdist(x.double(), y.double()), rtol=1e-5, atol=1e-5)
    ix, iy = 1 / x.norm(dim=1), 1 / y.norm(dim=1)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_COSINE, ix.to(DEV), iy.to(DEV)).cpu().double()
    ref = (x.double() / x.double().norm(dim=1, keepdim=True)) @ (y.double() / y.double().norm(dim=1, keepdim=True)).T
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_big_reductions():
    n, m, d = 4100, 4097, 96
    x, y = _xy(n, m, d, 2)
    xd, yd = x.to(DEV), y.to(DEV)
    dot = x.double() @ y.double().T
    part = ops.gemm_nt(xd, yd, ops.GEMM_POLY_SUM, scale=1 / d, coef=1.0, degree=3).cpu()
    torch.testing.assert_close(part.sum(), ((dot / d + 1) ** 3).sum(), rtol=1e-5, atol=1e-3)
    ix, iy = 1 / x.norm(dim=1), 1 / y.norm(dim=1)
    rmin = ops.gemm_nt(xd, yd, ops.GEMM_ROW_MIN, ix.to(DEV), iy.to(DEV)).cpu().min(-1).values.double()
    cos = dot * ix.double()[:, None] * iy.double()[None]
    torch.testing.assert_close(rmin, (1 - cos.abs()).min(1).values, rtol=1e-5, atol=1e-5)
    rsum = ops.gemm_nt(xd, yd, ops.GEMM_ROW_SUM, scale=0.25).cpu().sum(-1).double()
    torch.testing.assert_close(rsum, 0.25 * dot.sum(1), rtol=1e-4, atol=1e-2)
    rmax, cmax = ops.gemm_row_col_max(xd[None], yd[None], scale=0.5)
    torch.testing.assert_close(rmax[0].cpu().double(), 0.5 * dot.max(1).values, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(cmax[0].cpu().double(), 0.5 * dot.max(0).values, rtol=1e-5, atol=1e-4)


def test_big_batched_and_gathered():
    g = torch.Generator().manual_seed(3)
    xb, yb = torch.randn(8, 1024, 256, generator=g), torch.randn(8, 1280, 256, generator=g)
    out = ops.gemm_nt(xb.to(DEV), yb.to(DEV), ops.GEMM_STORE).cpu().double()
    torch.testing.assert_close(out, xb.double() @ yb.double().transpose(1, 2), rtol=1e-5, atol=2e-3)
    feats = torch.randn(4096, 256, generator=g)
    ix = torch.randint(0, 4096, (8, 1024), generator=g, dtype=torch.int32)
    iy = torch.randint(0, 4096, (8, 1024), generator=g, dtype=torch.int32)
    part = ops.gemm_nt(feats.to(DEV), feats.to(DEV), ops.GEMM_POLY_SUM, scale=1 / 256, coef=1.0, degree=3,
                       idx_x=ix.to(DEV), idx_y=iy.to(DEV)).cpu()
    fx, fy = feats.double()[ix.long()], feats.double()[iy.long()]
    ref = ((fx @ fy.transpose(1, 2) / 256 + 1) ** 3).sum((1, 2))
    torch.testing.assert_close(part.sum(-1), ref, rtol=1e-5, atol=1e-2)
