"""Euclidean distance precision on the fp64 matrix-core path vs the reference's fp64 formula
(``F/pairwise/euclidean.py:35-44``), on near-duplicate rows where an fp32 GEMM loses the cancellation."""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.pairwise import pairwise_euclidean_distance

pytestmark = pytest.mark.gpu


def _ref(x, y, zd):
    x64, y64 = x.double(), y.double()
    d = x64.pow(2).sum(1, keepdim=True) + y64.pow(2).sum(1) - 2 * x64 @ y64.T
    if zd:
        d.fill_diagonal_(0)
    return d.clamp(min=0).sqrt()


@pytest.mark.parametrize("n,m,d", [(300, 257, 64), (1024, 1024, 512), (129, 70, 33)])
def test_near_duplicate_rows(n, m, d):
    g = torch.Generator().manual_seed(n + d)
    base = torch.randn(m, d, generator=g) * 10
    y = base
    x = torch.cat([base[: min(n, m)] + 1e-3 * torch.randn(min(n, m), d, generator=g),
                   torch.randn(max(n - m, 0), d, generator=g)])[:n]
    got = pairwise_euclidean_distance(x.cuda(), y.cuda()).cpu()
    ref = _ref(x, y, False)
    rel = ((got.double() - ref).abs() / ref.clamp(min=1e-30)).max().item()
    assert rel <= 1e-6, rel


def test_self_distance_zero_diag_and_dtypes():
    g = torch.Generator().manual_seed(7)
    x = torch.randn(500, 96, generator=g) * 100
    # separation 1e-8 of |x|^2 (the fp64 formula's own rounding, ~1e-16 |x|^2, stays far below the 1e-6 bound; at
    # 1e-12 both the reference's and our fp64 evaluations carry ~1e-4 relative noise of their own)
    x[1] = x[0] + 1e-2
    got = pairwise_euclidean_distance(x.cuda()).cpu()
    ref = _ref(x, x, True)
    assert torch.isfinite(got).all()
    assert torch.allclose(got.double(), ref, rtol=1e-6, atol=0)
    for dt in (torch.float16, torch.bfloat16, torch.float64):
        xd = x[:, :64].to(dt) / 100
        out = pairwise_euclidean_distance(xd.cuda(), zero_diagonal=False).cpu()
        assert out.dtype == dt
        r = _ref(xd.double(), xd.double(), False)
        assert torch.allclose(out.double(), r, rtol=1e-2 if dt != torch.float64 else 1e-6, atol=1e-2)


def test_euclid_op_matches_cpu_path():
    g = torch.Generator().manual_seed(3)
    x, y = torch.randn(200, 48, generator=g), torch.randn(131, 48, generator=g)
    got = ops.euclid_f64(x.cuda(), y.cuda(), False, sqrt=False).cpu()
    ref = ops.euclid_f64(x, y, False, sqrt=False)
    assert torch.allclose(got, ref, rtol=1e-6, atol=1e-6)
