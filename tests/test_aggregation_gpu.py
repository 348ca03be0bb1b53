"""Fused aggregator update kernel (``csrc/common/aggregate.hip``) vs fp64 PyTorch formulas of the reference's
semantics (reference ``S/aggregation.py:75-105``: NaNs dropped for ignore / warn, x and w imputed for a float
strategy, RuntimeError for error)."""
import warnings

import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _expected(kind, x, w, strategy):
    w = torch.ones_like(x, dtype=torch.float64) if w is None else torch.broadcast_to(w.double(), x.shape)
    x, w = x.double().reshape(-1), w.reshape(-1).clone()
    nan = torch.isnan(x) | torch.isnan(w)
    if isinstance(strategy, float):
        x = x.clone()
        x[nan], w[nan] = strategy, strategy
    else:
        x, w = x[~nan], w[~nan]
    if kind == "sum":
        return (x * w).sum()
    if kind == "mean":
        return (x * w).sum() / w.sum()
    if x.numel() == 0:
        return torch.tensor(float("-inf") if kind == "max" else float("inf"), dtype=torch.float64)
    return x.max() if kind == "max" else x.min()


_CLS = {"sum": tm.SumMetric, "mean": tm.MeanMetric, "max": tm.MaxMetric, "min": tm.MinMetric}


@pytest.mark.parametrize("kind", ["sum", "mean", "max", "min"])
@pytest.mark.parametrize("n", [1, 7, 1000, 3_000_001])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
@pytest.mark.parametrize("strategy", ["ignore", 2.5])
def test_aggregators_match_fp64(kind, n, dtype, strategy):
    assert ops.native_available()
    g = torch.Generator().manual_seed(n)
    batches = [torch.randn(n, generator=g).to(dtype) for _ in range(3)]
    batches[1][:: max(1, n // 5)] = float("nan")
    m = _CLS[kind](nan_strategy=strategy).to(DEV)
    for b in batches:
        m.update(b.to(DEV))
    got = m.compute().cpu().double()
    if kind == "sum":
        exp = sum(_expected("sum", b, None, strategy) for b in batches)
    elif kind == "mean":
        cat = torch.cat(batches)
        exp = _expected("mean", cat, None, strategy)
    else:
        exp = _expected(kind, torch.cat(batches), None, strategy)
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-5 * max(1.0, n ** 0.5))


@pytest.mark.parametrize("wshape", ["scalar_py", "scalar_t", "full", "bcast"])
def test_mean_weights(wshape):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 33, generator=g)
    x[3, 5] = float("nan")
    if wshape == "scalar_py":
        w = 0.5
    elif wshape == "scalar_t":
        w = torch.tensor(3.0)
    elif wshape == "full":
        w = torch.rand(64, 33, generator=g)
        w[10, 1] = float("nan")
    else:
        w = torch.rand(33, generator=g)
    m = tm.MeanMetric(nan_strategy="ignore").to(DEV)
    m.update(x.to(DEV), w.to(DEV) if isinstance(w, torch.Tensor) else w)
    ref = tm.MeanMetric(nan_strategy="ignore")
    ref.update(x, w)
    torch.testing.assert_close(m.compute().cpu(), ref.compute(), rtol=1e-6, atol=1e-6)
    wt = w if isinstance(w, torch.Tensor) else torch.tensor(w)
    torch.testing.assert_close(m.compute().cpu().double(), _expected("mean", x, wt, "ignore"), rtol=1e-6, atol=1e-6)


def test_warn_and_error_strategies():
    x = torch.tensor([1.0, float("nan"), 3.0], device=DEV)
    m = tm.SumMetric(nan_strategy="warn").to(DEV)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        m.update(x)  # ROCm: no host sync in update, the warning bit is raised on the device
    with pytest.warns(UserWarning, match="Encountered `nan` values in tensor"):
        assert float(m.compute()) == 4.0
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        m.update(torch.ones(3, device=DEV))  # no NaN: the bit was consumed by the previous compute
        assert float(m.compute()) == 7.0
    f = tm.MeanMetric(nan_strategy="warn").to(DEV)
    with pytest.warns(UserWarning, match="Encountered `nan` values in tensor"):
        assert float(f(x)) == 2.0  # forward: the batch compute emits it (reference T/bases/test_aggregation.py:112)
    e = tm.MeanMetric(nan_strategy="error").to(DEV)
    e.update(x)
    with pytest.raises(RuntimeError, match="Encountered `nan` values in tensor"):
        e.compute()
    e.reset()
    e.update(torch.ones(4, device=DEV))
    assert float(e.compute()) == 1.0


def test_all_nan_ignored_keeps_state():
    x = torch.full((5,), float("nan"), device=DEV)
    mx = tm.MaxMetric(nan_strategy="ignore").to(DEV)
    mx.update(torch.tensor([2.0], device=DEV))
    mx.update(x)
    assert float(mx.compute()) == 2.0
    mean = tm.MeanMetric(nan_strategy="ignore").to(DEV)
    mean.update(x)
    assert torch.isnan(mean.compute())


def test_int_inputs_python_numbers_and_fp64_state():
    s = tm.SumMetric().to(DEV)
    s.update(torch.arange(10, device=DEV))
    s.update(2.5)
    assert float(s.compute()) == 47.5
    d = tm.MeanMetric().to(DEV).set_dtype(torch.float64)
    d.update(torch.tensor([1e-9, 1.0], dtype=torch.float64, device=DEV))
    assert d.compute().dtype == torch.float64
    assert float(d.compute()) == pytest.approx((1e-9 + 1.0) / 2, rel=1e-15)


def test_forward_and_deterministic():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2_000_000, generator=g).to(DEV)
    outs = []
    for _ in range(2):
        m = tm.MeanMetric().to(DEV)
        bv = m(x)
        m(x * 2)
        outs.append((bv.cpu(), m.compute().cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    torch.testing.assert_close(outs[0][0].double(), x.double().mean().cpu(), rtol=1e-6, atol=1e-7)


def test_grad_input_takes_autograd_path():
    x = torch.randn(16, device=DEV, requires_grad=True)
    m = tm.SumMetric().to(DEV)
    out = m(x)  # forward enables grad for the batch value (as the reference): the autograd path runs
    out.backward()
    assert torch.equal(x.grad, torch.ones_like(x))
