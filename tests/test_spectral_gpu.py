"""SAM / ERGAS on the one-pass spectral kernels (``csrc/image/spectral.hip``) vs the reference formulas
(``F/image/sam.py:56-83``, ``F/image/ergas.py:57-71``) evaluated with torch ops on the CPU."""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd.functional import error_relative_global_dimensionless_synthesis as ergas
from torchmetrics_amd.functional import spectral_angle_mapper as sam

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _sam_ref(p, t, reduction):
    p, t = p.double(), t.double()
    a = torch.clamp((p * t).sum(1) / (p.norm(dim=1) * t.norm(dim=1)), -1, 1).acos()
    return {"elementwise_mean": a.mean(), "sum": a.sum(), "none": a, None: a}[reduction]


def _ergas_ref(p, t, ratio, reduction):
    p, t = p.double(), t.double()
    b, c, h, w = p.shape
    pp, tt = p.reshape(b, c, -1), t.reshape(b, c, -1)
    rmse = torch.sqrt(((pp - tt) ** 2).sum(2) / (h * w))
    s = 100 * ratio * torch.sqrt(torch.sum((rmse / tt.mean(2)) ** 2, 1) / c)
    return {"elementwise_mean": s.mean(), "sum": s.sum(), "none": s, None: s}[reduction]


@pytest.mark.parametrize("shape", [(4, 3, 16, 16), (2, 31, 67, 45), (1, 2, 300, 301)])
@pytest.mark.parametrize("reduction", ["elementwise_mean", "sum", "none"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_sam_matches_reference(shape, reduction, dtype):
    g = torch.Generator().manual_seed(sum(shape))
    p, t = torch.rand(shape, generator=g).to(dtype), torch.rand(shape, generator=g).to(dtype)
    got = sam(p.to(DEV), t.to(DEV), reduction=reduction).cpu()
    assert got.dtype == dtype
    # fp32: acos near cos = 1 turns the cosine's last-bit rounding into up to sqrt(2 eps) ~ 5e-4 of angle for nearly
    # parallel vectors -- the reference's fp32 evaluation carries the same error; compared against fp64 here
    atol = {torch.float32: 1e-3, torch.float64: 1e-10, torch.bfloat16: 3e-2}[dtype]
    rtol = {torch.float32: 1e-4, torch.float64: 1e-10, torch.bfloat16: 2e-2}[dtype]
    torch.testing.assert_close(got.double(), _sam_ref(p, t, reduction), rtol=rtol, atol=atol)


def test_sam_zero_vector_is_nan_like_reference():
    p = torch.rand(2, 3, 4, 4)
    p[0, :, 1, 2] = 0
    t = torch.rand(2, 3, 4, 4)
    got = sam(p.to(DEV), t.to(DEV), reduction="none").cpu()
    ref = _sam_ref(p, t, "none")
    assert torch.isnan(got[0, 1, 2]) and torch.isnan(ref[0, 1, 2])
    torch.testing.assert_close(got.double(), ref, equal_nan=True, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape", [(4, 3, 16, 16), (3, 5, 257, 129), (1, 1, 1024, 1024)])
@pytest.mark.parametrize("reduction", ["elementwise_mean", "sum", "none"])
def test_ergas_matches_reference(shape, reduction):
    g = torch.Generator().manual_seed(shape[2])
    p, t = torch.rand(shape, generator=g) + 0.1, torch.rand(shape, generator=g) + 0.1
    got = ergas(p.to(DEV), t.to(DEV), ratio=4, reduction=reduction).cpu()
    torch.testing.assert_close(got.double(), _ergas_ref(p, t, 4, reduction), rtol=1e-5, atol=1e-5)


def test_modules_and_autograd_path():
    g = torch.Generator().manual_seed(0)
    p, t = torch.rand(6, 4, 32, 32, generator=g), torch.rand(6, 4, 32, 32, generator=g)
    m = tm.image.SpectralAngleMapper().to(DEV)
    e = tm.image.ErrorRelativeGlobalDimensionlessSynthesis().to(DEV)
    for i in range(0, 6, 2):
        m.update(p[i:i + 2].to(DEV), t[i:i + 2].to(DEV))
        e.update(p[i:i + 2].to(DEV), t[i:i + 2].to(DEV))
    torch.testing.assert_close(m.compute().cpu().double(), _sam_ref(p, t, "elementwise_mean"), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(e.compute().cpu().double(), _ergas_ref(p, t, 4, "elementwise_mean"), rtol=1e-5, atol=1e-5)
    # gradients still flow (the kernels are bypassed when autograd needs the graph)
    pg = p[:2].to(DEV).requires_grad_()
    sam(pg, t[:2].to(DEV)).backward()
    assert pg.grad is not None and torch.isfinite(pg.grad).all()
