"""Row + column max epilogue of the MFMA GEMM (``csrc/pairwise/gemm_nt.hip`` ROW_COL_MAX) and BERTScore's greedy
matching built on it, vs fp64 PyTorch."""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.text.bert import _greedy_match
from tests.helpers import assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize(("b", "n", "m", "d"), [(1, 1, 1, 4), (3, 37, 129, 64), (5, 128, 128, 768), (2, 300, 257, 1024),
                                               (64, 12, 30, 384)])
def test_row_col_max_vs_fp64(b, n, m, d):
    g = torch.Generator().manual_seed(n * m)
    x = torch.randn(b, n, d, generator=g)
    y = torch.randn(b, m, d, generator=g)
    rows, cols = ops.gemm_row_col_max(x.cuda(), y.cuda(), scale=0.5)
    dot = torch.bmm(x.double(), y.double().transpose(1, 2)) * 0.5
    assert_close(rows.cpu().double(), dot.amax(2), atol=1e-3, rtol=1e-5)
    assert_close(cols.cpu().double(), dot.amax(1), atol=1e-3, rtol=1e-5)
    r_cpu, c_cpu = ops.gemm_row_col_max(x, y, scale=0.5)  # host contract, same partial layout
    assert_close(r_cpu.double(), dot.amax(2), atol=1e-3, rtol=1e-5)
    assert_close(c_cpu.double(), dot.amax(1), atol=1e-3, rtol=1e-5)


def test_bertscore_greedy_match_gpu_vs_cpu():
    g = torch.Generator().manual_seed(0)
    n, layers, p, r, d = 6, 2, 23, 31, 128
    pe = torch.nn.functional.normalize(torch.randn(n, layers, p, d, generator=g), dim=-1)
    te = torch.nn.functional.normalize(torch.randn(n, layers, r, d, generator=g), dim=-1)
    pe[:, :, -3:] = 0  # padding tokens carry zero embeddings
    pw = torch.rand(n, p, generator=g)
    tw = torch.rand(n, r, generator=g)
    got = _greedy_match(pe.cuda(), te.cuda(), pw.cuda(), tw.cuda())
    want = _greedy_match(pe, te, pw, tw)
    for a, w in zip(got, want):
        assert_close(a.cpu(), w, atol=1e-5, rtol=1e-5)
