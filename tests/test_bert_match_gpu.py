"""BERTScore greedy matching on ROCm (``csrc/text/bert_match.hip`` for <= 128 tokens a side, the 128-tile MFMA GEMM
epilogue beyond) against the plain PyTorch fp32 formulation (``matmul`` + ``amax``) of the same function."""
import pytest
import torch

from torchmetrics_amd.functional.text.bert import _greedy_match

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("p,r", [(7, 9), (40, 33), (64, 64), (65, 17), (128, 100), (150, 131)])
@pytest.mark.parametrize("d", [768, 30])
def test_greedy_match_matches_torch(p, r, d):
    g = torch.Generator().manual_seed(p * 1000 + r + d)
    n, nl = 5, 2
    pe = torch.nn.functional.normalize(torch.randn(n, nl, p, d, generator=g), dim=-1)
    te = torch.nn.functional.normalize(torch.randn(n, nl, r, d, generator=g), dim=-1)
    pw = torch.rand(n, p, generator=g)
    tw = torch.rand(n, r, generator=g)
    got = _greedy_match(pe.to(DEV), te.to(DEV), pw.to(DEV), tw.to(DEV))
    cos = torch.matmul(pe.double(), te.double().transpose(-1, -2))
    exp_p = (cos.amax(dim=3) * pw[:, None, :].double()).sum(-1)
    exp_r = (cos.amax(dim=2) * tw[:, None, :].double()).sum(-1)
    torch.testing.assert_close(got[0].cpu().double(), exp_p, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got[1].cpu().double(), exp_r, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("p,r,d", [(7, 9, 768), (40, 33, 768), (128, 100, 64), (65, 17, 30), (150, 131, 768)])
def test_greedy_match_16bit_embeddings(dtype, p, r, d):
    """bf16 / fp16 embeddings run the 16-bit matcher (no fp32 upcast): the maxima equal those of an fp64 matmul of
    the same 16-bit values rounded to the embedding dtype -- the reference's einsum output dtype
    (F/text/bert.py:159)."""
    from torchmetrics_amd import ops

    g = torch.Generator().manual_seed(p * 7 + r + d)
    n, nl = 4, 2
    pe = torch.nn.functional.normalize(torch.randn(n, nl, p, d, generator=g), dim=-1).to(dtype)
    te = torch.nn.functional.normalize(torch.randn(n, nl, r, d, generator=g), dim=-1).to(dtype)
    pw = torch.rand(n, p, generator=g)
    tw = torch.rand(n, r, generator=g)
    if p <= 128 and r <= 128:
        rm, cm = ops.bert_rowcol_max(pe.reshape(n * nl, p, d).to(DEV), te.reshape(n * nl, r, d).to(DEV))
        cos = torch.matmul(pe.double(), te.double().transpose(-1, -2)).reshape(n * nl, p, r)
        tol = dict(rtol=0, atol=float(torch.finfo(dtype).eps))  # one rounding step of the 16-bit output
        torch.testing.assert_close(rm.cpu().double(), cos.amax(2).to(dtype).double(), **tol)
        torch.testing.assert_close(cm.cpu().double(), cos.amax(1).to(dtype).double(), **tol)
    got = _greedy_match(pe.to(DEV), te.to(DEV), pw.to(DEV), tw.to(DEV))
    cos = torch.matmul(pe.double(), te.double().transpose(-1, -2)).to(dtype).double()
    exp_p = (cos.amax(dim=3) * pw[:, None, :].double()).sum(-1)
    exp_r = (cos.amax(dim=2) * tw[:, None, :].double()).sum(-1)
    torch.testing.assert_close(got[0].cpu().double(), exp_p, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(got[1].cpu().double(), exp_r, rtol=1e-2, atol=1e-2)
