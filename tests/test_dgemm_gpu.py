"""fp64 matrix-core GEMM / power-iteration GEMV (``csrc/image/dgemm.hip``) against plain PyTorch fp64 ops."""
import pytest
import torch

from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("shape", [(2048, 2048, 2048), (256, 256, 256), (130, 77, 200), (1, 5, 3), (300, 129, 64)])
def test_dgemm_matches_torch(shape):
    m, k, n = shape
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g, dtype=torch.float64)
    b = torch.randn(k, n, generator=g, dtype=torch.float64)
    c0 = torch.randn(m, n, generator=g, dtype=torch.float64)
    out = torch.empty(m, n, dtype=torch.float64, device=DEV)
    ops.dgemm(a.to(DEV), b.to(DEV), out, alpha=-0.75, beta=1.5, cin=c0.to(DEV), diag=2.0)
    ref = -0.75 * (a @ b) + 1.5 * c0 + 2.0 * torch.eye(m, n, dtype=torch.float64)
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-12, atol=1e-11 * k)


def test_dgemm_batched_two_problems_and_no_cin():
    g = torch.Generator().manual_seed(3)
    y, w, z = (torch.randn(512, 512, generator=g, dtype=torch.float64) for _ in range(3))
    yd, wd, zd = y.to(DEV), w.to(DEV), z.to(DEV)
    y2, z2 = torch.empty_like(yd), torch.empty_like(zd)
    ops.dgemm([yd, wd], [wd, zd], [y2, z2], alpha=[0.3, 0.3], beta=[1.2, 1.2], cin=[yd, zd])
    torch.testing.assert_close(y2.cpu(), 0.3 * (y @ w) + 1.2 * y, rtol=1e-12, atol=1e-10)
    torch.testing.assert_close(z2.cpu(), 0.3 * (w @ z) + 1.2 * z, rtol=1e-12, atol=1e-10)
    p = torch.empty_like(yd)
    ops.dgemm(yd, zd, p)
    torch.testing.assert_close(p.cpu(), y @ z, rtol=1e-12, atol=1e-10)
    p2 = torch.empty_like(yd)
    ops.dgemm(yd, zd, p2)
    assert torch.equal(p, p2)  # fixed accumulation order


def test_dgemv4_power_step():
    d = 1000
    g = torch.Generator().manual_seed(5)
    a = torch.randn(d, d, generator=g, dtype=torch.float64) / d
    v = torch.rand(d, 4, generator=g, dtype=torch.float64)
    nb = ops.dgemv4_blocks(d)
    w1 = torch.empty(d, 4, dtype=torch.float64, device=DEV)
    p1 = torch.empty(nb, 4, dtype=torch.float64, device=DEV)
    dummy = torch.zeros(4, dtype=torch.float64, device=DEV)
    ops.dgemv4_resid(a.to(DEV), v.to(DEV), dummy, False, w1, p1)
    ref1 = v - a @ v
    torch.testing.assert_close(w1.cpu(), ref1, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(p1.sum(0).cpu(), (ref1 ** 2).sum(0), rtol=1e-12, atol=1e-12)
    w2 = torch.empty_like(w1)
    p2 = torch.empty_like(p1)
    ops.dgemv4_resid(a.to(DEV), w1, p1, True, w2, p2)
    vn = ref1 / ref1.norm(dim=0)
    torch.testing.assert_close(w2.cpu(), vn - a @ vn, rtol=1e-11, atol=1e-12)
