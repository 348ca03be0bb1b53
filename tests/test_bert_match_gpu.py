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
