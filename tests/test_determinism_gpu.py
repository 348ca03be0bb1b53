"""Run-to-run determinism of the GPU kernels (SURVEY §5 "determinism").

Integer states (confusion matrices, stat scores, binned curves, histograms) are accumulated with 64-bit integer
atomics, so their results are bitwise reproducible whatever the block schedule.  Floating-point reductions with a
fixed order (regression moments: per-block partials folded in block order; FID's fp64 SYRK; fused compute kernels)
are bitwise reproducible too.  The float-atomic kernels (calibration bins across blocks) are order-dependent by
design; their run-to-run spread is bounded here instead of asserted zero.
"""
import pytest
import torch

import torchmetrics_amd.classification as C
import torchmetrics_amd.regression as R
from torchmetrics_amd.image import FrechetInceptionDistance

pytestmark = pytest.mark.gpu


def _run_twice(make, feed):
    out = []
    for _ in range(2):
        m = make().cuda()
        feed(m)
        out.append((m.compute(), {k: v.clone() if isinstance(v, torch.Tensor) else v
                                  for k, v in m.metric_state.items()}))
    return out


def _same(a, b):
    if isinstance(a, (list, tuple)):
        return all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return all(_same(a[k], b[k]) for k in a)
    return torch.equal(a, b)


def _cls_feed(m):
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(5):
        m.update(torch.randn(20000, 10, device="cuda", generator=g).to(torch.bfloat16),
                 torch.randint(0, 10, (20000,), device="cuda", generator=g))


@pytest.mark.parametrize("make", [
    lambda: C.MulticlassConfusionMatrix(10), lambda: C.MulticlassStatScores(10, average=None),
    lambda: C.MulticlassAUROC(10, thresholds=50), lambda: C.MulticlassAccuracy(10),
    lambda: C.MulticlassCohenKappa(10)])
def test_integer_state_metrics_bitwise_reproducible(make):
    (r1, s1), (r2, s2) = _run_twice(make, _cls_feed)
    assert _same(r1, r2) and _same(s1, s2)


def _reg_feed(m):
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(4):
        p = torch.randn(100000, device="cuda", generator=g)
        m.update(p, p + 0.1 * torch.randn(100000, device="cuda", generator=g))


@pytest.mark.parametrize("make", [R.MeanSquaredError, R.PearsonCorrCoef, R.R2Score, R.ExplainedVariance,
                                  R.MeanAbsoluteError])
def test_fixed_order_float_reductions_bitwise_reproducible(make):
    (r1, s1), (r2, s2) = _run_twice(make, _reg_feed)
    assert _same(r1, r2) and _same(s1, s2)


def test_fid_syrk_bitwise_reproducible():
    class _Id(torch.nn.Module):
        num_features = 256

        def forward(self, x):
            return x

    def feed(m):
        g = torch.Generator(device="cuda").manual_seed(2)
        for real in (True, False):
            for _ in range(3):
                m.update(torch.randn(5000, 256, device="cuda", generator=g), real=real)

    (r1, s1), (r2, s2) = _run_twice(lambda: FrechetInceptionDistance(feature=_Id()), feed)
    assert _same(r1, r2) and _same(s1, s2)


def test_float_atomic_calibration_bins_spread_is_tiny():
    def feed(m):
        g = torch.Generator(device="cuda").manual_seed(3)
        for _ in range(3):
            m.update(torch.randn(400000, 5, device="cuda", generator=g),
                     torch.randint(0, 5, (400000,), device="cuda", generator=g))

    (r1, _), (r2, _) = _run_twice(lambda: C.MulticlassCalibrationError(5, n_bins=15), feed)
    assert abs(float(r1) - float(r2)) <= 1e-6
