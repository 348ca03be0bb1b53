"""16-bit MFMA NT-GEMM (``gemm_nt_h16_kernel``: v_mfma_f32_32x32x16_{bf16,f16}, fp32 accumulate) against a plain
PyTorch fp32 GEMM of the same 16-bit values (the products are exact in fp32, only the summation order differs): every
epilogue, both tile sizes (128 x 128 for small problems, 256 x 256 once the tiles fill the chip), K not a multiple of
the 64-element k-chunk, partial tiles, batched and row-gathered operands, 16-bit outputs, and the pairwise functionals
that route bf16 / fp16 here (reference F/pairwise/linear.py:23, cosine.py:24-46: GEMM in the input dtype)."""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
DT = [torch.bfloat16, torch.float16]


def _xy(n, m, d, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    return ((torch.randn(n, d, generator=g)).to(dtype), (torch.randn(m, d, generator=g) * 0.5 + 0.1).to(dtype))


def _tol(d):
    return dict(rtol=2e-5, atol=2e-5 * d ** 0.5)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,m,d", [(300, 200, 72), (128, 128, 64), (1000, 777, 200), (4100, 4097, 96),
                                   (4096, 4096, 8), (4097, 4096, 520)])
def test_h16_store(dtype, n, m, d):
    x, y = _xy(n, m, d, dtype)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_STORE, scale=0.5)
    assert out.dtype == torch.float32
    ref = 0.5 * (x.double() @ y.double().T)
    torch.testing.assert_close(out.cpu().double(), ref, **_tol(d))
    o16 = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_STORE, scale=0.5, out_dtype=dtype)
    assert o16.dtype == dtype
    assert torch.equal(o16.cpu(), out.cpu().to(dtype))  # the epilogue rounds exactly as a cast of the fp32 result


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,m,d", [(333, 257, 136), (4100, 4097, 96)])
def test_h16_cosine_euclid(dtype, n, m, d):
    x, y = _xy(n, m, d, dtype, 1)
    xd, yd = x.double(), y.double()
    ix, iy = 1 / xd.norm(dim=1), 1 / yd.norm(dim=1)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_COSINE, ix.float().to(DEV), iy.float().to(DEV))
    ref = (xd @ yd.T) * ix[:, None] * iy[None]
    torch.testing.assert_close(out.cpu().double(), ref, rtol=1e-5, atol=1e-5)
    nx, ny = (xd * xd).sum(1), (yd * yd).sum(1)
    out = ops.gemm_nt(x.to(DEV), y.to(DEV), ops.GEMM_EUCLID, nx.float().to(DEV), ny.float().to(DEV))
    torch.testing.assert_close(out.cpu().double(), torch.cdist(xd, yd), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,m,d", [(517, 300, 64), (4100, 4097, 96)])
def test_h16_reductions(dtype, n, m, d):
    x, y = _xy(n, m, d, dtype, 2)
    xd, yd = x.to(DEV), y.to(DEV)
    dot = x.double() @ y.double().T
    part = ops.gemm_nt(xd, yd, ops.GEMM_POLY_SUM, scale=1 / d, coef=1.0, degree=3).cpu()
    torch.testing.assert_close(part.sum(), ((dot / d + 1) ** 3).sum(), rtol=1e-5, atol=1e-2)
    ix, iy = 1 / x.double().norm(dim=1), 1 / y.double().norm(dim=1)
    rmin = ops.gemm_nt(xd, yd, ops.GEMM_ROW_MIN, ix.float().to(DEV), iy.float().to(DEV)).cpu().min(-1).values
    cos = dot * ix[:, None] * iy[None]
    torch.testing.assert_close(rmin.double(), (1 - cos.abs()).min(1).values, rtol=1e-5, atol=1e-5)
    rsum = ops.gemm_nt(xd, yd, ops.GEMM_ROW_SUM, scale=0.25).cpu().sum(-1).double()
    torch.testing.assert_close(rsum, 0.25 * dot.sum(1), rtol=1e-4, atol=1e-2)
    rmax, cmax = ops.gemm_row_col_max(xd[None], yd[None], scale=0.5)
    torch.testing.assert_close(rmax[0].cpu().double(), 0.5 * dot.max(1).values, **_tol(d))
    torch.testing.assert_close(cmax[0].cpu().double(), 0.5 * dot.max(0).values, **_tol(d))


@pytest.mark.parametrize("dtype", DT)
def test_h16_batched_gathered_zero_diag(dtype):
    g = torch.Generator().manual_seed(3)
    xb, yb = torch.randn(3, 300, 136, generator=g).to(dtype), torch.randn(3, 260, 136, generator=g).to(dtype)
    out = ops.gemm_nt(xb.to(DEV), yb.to(DEV), ops.GEMM_STORE, zero_diagonal=True).cpu().double()
    ref = xb.double() @ yb.double().transpose(1, 2)
    ref[:, torch.arange(260), torch.arange(260)] = 0
    torch.testing.assert_close(out, ref, **_tol(136))
    feats = torch.randn(2000, 128, generator=g).to(dtype)
    ix = torch.randint(0, 2000, (4, 500), generator=g, dtype=torch.int32)
    iy = torch.randint(0, 2000, (4, 400), generator=g, dtype=torch.int32)
    part = ops.gemm_nt(feats.to(DEV), feats.to(DEV), ops.GEMM_POLY_SUM, scale=1 / 128, coef=1.0, degree=3,
                       idx_x=ix.to(DEV), idx_y=iy.to(DEV)).cpu()
    fx, fy = feats.double()[ix.long()], feats.double()[iy.long()]
    torch.testing.assert_close(part.sum(-1), ((fx @ fy.transpose(1, 2) / 128 + 1) ** 3).sum((1, 2)), rtol=1e-5,
                               atol=1e-2)


@pytest.mark.parametrize("dtype", DT)
def test_pairwise_functionals_16bit(dtype):
    x, y = _xy(700, 500, 96, dtype, 4)
    lin = tm.functional.pairwise_linear_similarity(x.to(DEV), y.to(DEV))
    assert lin.dtype == dtype
    torch.testing.assert_close(lin.cpu().float(), (x.float() @ y.float().T).to(dtype).float(), rtol=1e-2, atol=1e-2)
    cos = tm.functional.pairwise_cosine_similarity(x.to(DEV), zero_diagonal=False)
    assert cos.dtype == dtype
    xn = x.double() / x.double().norm(dim=1, keepdim=True)
    torch.testing.assert_close(cos.cpu().double(), xn @ xn.T, rtol=1e-2, atol=1e-2)
    cz = tm.functional.pairwise_cosine_similarity(x.to(DEV))  # y defaults to x, zero diagonal
    assert torch.count_nonzero(torch.diagonal(cz)) == 0


def test_h16_no_upcast_kernel():
    """bf16 operands reach the 16-bit kernel directly: no fp32 copy of the operands is made."""
    x, y = _xy(4096, 4096, 512, torch.bfloat16)
    xd, yd = x.to(DEV), y.to(DEV)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    before = torch.cuda.memory_allocated()
    out = ops.gemm_nt(xd, yd, ops.GEMM_STORE, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    peak_extra = torch.cuda.max_memory_allocated() - before
    assert out.dtype == torch.bfloat16
    assert peak_extra <= out.numel() * 2 + (1 << 20)  # only the bf16 output (an fp32 copy of x would be 8 MB)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("d", [512, 100, 8])
def test_row_norms_kernel(dtype, d):
    """csrc/pairwise/gemm_nt.hip row_norms (one wave per row, fp32 accumulation) against an fp64 torch reference;
    two operands from one launch."""
    g = torch.Generator().manual_seed(d)
    x = torch.randn(1037, d, generator=g).to(dtype)
    y = torch.randn(77, d, generator=g).to(dtype)
    ref_x = x.double().pow(2).sum(1)
    ref_y = y.double().pow(2).sum(1)
    sq = ops.row_norms(x.to(DEV)).cpu().double()
    torch.testing.assert_close(sq, ref_x, rtol=1e-5, atol=1e-6)
    ix, iy = ops.row_norms(x.to(DEV), inverse=True, y=y.to(DEV))
    torch.testing.assert_close(ix.cpu().double(), 1 / ref_x.sqrt(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(iy.cpu().double(), 1 / ref_y.sqrt(), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("n,m,d,shift", [(300, 200, 100, 0), (257, 131, 77, 0), (300, 200, 72, 1), (129, 65, 5, 0),
                                         (1000, 600, 130, 3), (64, 64, 1, 0)])
def test_h16_any_width_and_alignment_stays_16bit(dtype, n, m, d, shift):
    """Rows that are not 16-byte aligned (D % 8 != 0, or a base address off by ``shift`` elements) run the 16-bit
    kernel with narrower DMA lanes and in-kernel K padding (csrc/pairwise/gemm_nt.hip GRAN): no fp32 upcast copy, the
    same results as an fp64 GEMM of the 16-bit values, for the element-wise and the reduction epilogues."""
    x, y = _xy(n, m, d, dtype, 5)
    bx = torch.zeros(n * d + shift, dtype=dtype)
    by = torch.zeros(m * d + shift, dtype=dtype)
    bx[shift:] = x.reshape(-1)
    by[shift:] = y.reshape(-1)
    xd = bx.to(DEV)[shift:].view(n, d)
    yd = by.to(DEV)[shift:].view(m, d)
    assert xd.is_contiguous() and (shift == 0 or xd.data_ptr() % 16 != 0)
    calls = []
    real_float = torch.Tensor.float

    def spy(self, *a, **k):
        if self.is_cuda and self.dtype == dtype and self.dim() >= 2:
            calls.append(tuple(self.shape))
        return real_float(self, *a, **k)

    torch.Tensor.float = spy
    try:
        out = ops.gemm_nt(xd, yd, ops.GEMM_STORE)
        rows, cols = ops.gemm_row_col_max(xd[None], yd[None])
    finally:
        torch.Tensor.float = real_float
    assert not calls, f"operands upcast to fp32: {calls}"
    dot = x.double() @ y.double().T
    torch.testing.assert_close(out.cpu().double(), dot, **_tol(d))
    torch.testing.assert_close(rows[0].cpu().double(), dot.max(1).values, **_tol(d))
    torch.testing.assert_close(cols[0].cpu().double(), dot.max(0).values, **_tol(d))
    xx, yy = x.double(), y.double()
    nx, ny = (xx * xx).sum(1), (yy * yy).sum(1)
    e = ops.gemm_nt(xd, yd, ops.GEMM_EUCLID, nx.float().to(DEV), ny.float().to(DEV))
    torch.testing.assert_close(e.cpu().double(), torch.cdist(xx, yy), rtol=1e-4, atol=1e-4)
