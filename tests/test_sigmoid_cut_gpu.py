"""The binary / multilabel kernels decide the logit reading (`round(sigmoid(x)) > threshold`) as `x >= cut`
(``csrc/classification/stat_scores.hip`` ``sigmoid_cut``).  This holds because the device expression is
non-decreasing in x; checked here against the direct per-element expression on the device for EVERY bf16 and fp16
value and a dense fp32 sweep around each cut, at several thresholds."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _probe(x, thr, kind):
    from torchmetrics_amd import ops

    ops._ops()  # loads the extension
    return torch.ops.tm_amd.sigmoid_cut_probe(x.contiguous(), thr, kind).cpu()


@pytest.mark.parametrize("thr", [0.5, 0.3, 0.9, 0.999, 1e-4, 0.0, 1.0, -0.5, 2.0])
@pytest.mark.parametrize("dtype,kind", [(torch.bfloat16, 1), (torch.float16, 2)])
def test_cut_equals_direct_for_every_16bit_value(thr, dtype, kind):
    bits = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16)
    x = bits.view(dtype).float().cuda()
    out = _probe(x, thr, kind)
    direct, cut = out & 1, (out >> 1) & 1
    bad = (direct != cut).nonzero().flatten()
    assert bad.numel() == 0, (thr, x.cpu()[bad[:8]])


@pytest.mark.parametrize("thr", [0.5, 0.3, 0.9, 1e-3])
def test_cut_equals_direct_fp32_sweep(thr):
    import math

    c = math.log(thr / (1 - thr))
    base = torch.tensor([c], dtype=torch.float32)
    bits = base.view(torch.int32) + torch.arange(-200_000, 200_000, dtype=torch.int32)
    x = torch.cat([bits.view(torch.float32), torch.linspace(-100, 100, 200_001)]).cuda()
    out = _probe(x, thr, 0)
    assert torch.equal(out & 1, (out >> 1) & 1)
