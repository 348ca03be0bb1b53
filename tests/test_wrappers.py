"""Wrapper metrics: BootStrapper, ClasswiseWrapper, MinMaxMetric, MultioutputWrapper, MultitaskWrapper,
MetricTracker, FeatureShare (reference test model: ``T/wrappers``)."""
import numpy as np
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd.image import FrechetInceptionDistance, KernelInceptionDistance
from torchmetrics_amd.wrappers import FeatureShare
from torchmetrics_amd.wrappers.bootstrapping import _bootstrap_sampler
from tests.helpers import assert_close

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("strategy", ["poisson", "multinomial"])
def test_bootstrapper_matches_manual_resampling(device, strategy):
    p, t = torch.randn(200), torch.randn(200)
    torch.manual_seed(42)
    bs = tm.BootStrapper(tm.MeanSquaredError(), num_bootstraps=5, sampling_strategy=strategy, raw=True,
                         quantile=torch.tensor([0.05, 0.95], device=device)).to(device)
    bs.update(p.to(device), t.to(device))
    out = bs.compute()
    torch.manual_seed(42)
    vals = []
    for _ in range(5):
        idx = _bootstrap_sampler(200, strategy)
        vals.append(((p[idx] - t[idx]) ** 2).mean())
    vals = torch.stack(vals)
    assert_close(out["raw"], vals, atol=1e-5)
    assert_close(out["mean"], vals.mean(), atol=1e-5)
    assert_close(out["std"], vals.std(), atol=1e-5)
    assert out["quantile"].shape == (2,)


def test_bootstrapper_reference_docstring_values():
    """Golden value of reference ``S/wrappers/bootstrapping.py:76-86`` (same seed -> same replicates)."""
    torch.manual_seed(123)
    bootstrap = tm.BootStrapper(tm.MulticlassAccuracy(num_classes=5, average="micro"), num_bootstraps=20)
    bootstrap.update(torch.randint(5, (20,)), torch.randint(5, (20,)))
    out = bootstrap.compute()
    assert set(out) == {"mean", "std"}
    assert torch.allclose(out["mean"], torch.tensor(0.2205), atol=5e-5)
    assert torch.allclose(out["std"], torch.tensor(0.0859), atol=5e-5)


STAT_FAMILY = [tm.MulticlassAccuracy, tm.MulticlassPrecision, tm.MulticlassRecall, tm.MulticlassF1Score,
               tm.MulticlassSpecificity, tm.MulticlassHammingDistance, tm.MulticlassStatScores]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("cls", STAT_FAMILY)
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", "none"])
@pytest.mark.parametrize("strategy", ["poisson", "multinomial"])
def test_bootstrapper_batched_stat_family_matches_copies(device, cls, average, strategy):
    """The stacked one-kernel update / one-reduction compute equals computing every replicate copy on its own, and
    both equal replaying the same replicates through a fresh metric (ignore_index and label preds included)."""
    torch.manual_seed(3)
    base = cls(num_classes=4, average=average, ignore_index=2)
    bs = tm.BootStrapper(base, num_bootstraps=6, mean=False, std=False, raw=True, sampling_strategy=strategy)
    bs = bs.to(device)
    assert bs._stacked is not None
    batches = [(torch.randn(40, 4), torch.randint(4, (40,))), (torch.randint(4, (33,)), torch.randint(4, (33,)))]
    torch.manual_seed(11)
    for p, t in batches:
        bs.update(p.to(device), t.to(device))
    raw = bs.compute()["raw"].cpu()
    per_copy = torch.stack([m.compute() for m in bs.metrics]).cpu()
    torch.testing.assert_close(raw.float(), per_copy.float(), equal_nan=True)
    # replay the same replicates through fresh metrics
    torch.manual_seed(11)
    refs = [cls(num_classes=4, average=average, ignore_index=2) for _ in range(6)]
    for p, t in batches:
        for r in refs:
            idx = _bootstrap_sampler(len(t), strategy)
            if idx.numel():
                r.update(p[idx], t[idx])
    expect = torch.stack([r.compute() for r in refs])
    torch.testing.assert_close(raw.float(), expect.float(), equal_nan=True)


@pytest.mark.parametrize("device", DEVICES)
def test_bootstrapper_batched_flags_out_of_range_target(device):
    bs = tm.BootStrapper(tm.MulticlassAccuracy(num_classes=3), num_bootstraps=4).to(device)
    t = torch.tensor([0, 1, 2, 7])
    if device == "cpu":
        with pytest.raises(RuntimeError):
            bs.update(torch.randn(4, 3), t)
    else:
        bs.update(torch.randn(4, 3, device=device), t.to(device))
        with pytest.raises(RuntimeError):
            bs.compute()


def test_classwise_wrapper():
    m = tm.ClasswiseWrapper(tm.MulticlassAccuracy(num_classes=3, average=None), labels=["a", "b", "c"])
    p, t = torch.randn(20, 3), torch.randint(0, 3, (20,))
    out = m(p, t)
    assert set(out) == {"multiclassaccuracy_a", "multiclassaccuracy_b", "multiclassaccuracy_c"}
    ref = tm.functional.multiclass_accuracy(p, t, 3, average=None)
    assert_close(torch.stack([out[k] for k in sorted(out)]), ref)
    m2 = tm.ClasswiseWrapper(tm.MulticlassAccuracy(num_classes=3, average=None), prefix="acc-")
    assert set(m2(p, t)) == {"acc-0", "acc-1", "acc-2"}


def test_minmax():
    m = tm.MinMaxMetric(tm.MeanSquaredError())
    vals = []
    for i in range(4):
        p, t = torch.randn(10), torch.randn(10)
        m.update(p, t)
        out = m.compute()
        vals.append(out["raw"].item())
        assert out["max"].item() == pytest.approx(max(vals))
        assert out["min"].item() == pytest.approx(min(vals))


@pytest.mark.parametrize("device", DEVICES)
def test_multioutput(device):
    p, t = torch.randn(50, 3), torch.randn(50, 3)
    t[3, 1] = float("nan")
    m = tm.MultioutputWrapper(tm.MeanAbsoluteError(), num_outputs=3).to(device)
    m.update(p.to(device), t.to(device))
    res = m.compute()
    ref = []
    for j in range(3):
        keep = ~torch.isnan(t[:, j])
        ref.append((p[keep, j] - t[keep, j]).abs().mean())
    assert_close(res, torch.stack(ref), atol=1e-6)


def test_multitask():
    mt = tm.MultitaskWrapper({
        "cls": tm.BinaryAccuracy(),
        "reg": tm.MetricCollection([tm.MeanSquaredError(), tm.MeanAbsoluteError()]),
    })
    pc, tc = torch.rand(10), torch.randint(0, 2, (10,))
    pr, tr = torch.randn(10), torch.randn(10)
    mt.update({"cls": pc, "reg": pr}, {"cls": tc, "reg": tr})
    out = mt.compute()
    assert_close(out["cls"], tm.functional.binary_accuracy(pc, tc))
    assert_close(out["reg"]["MeanSquaredError"], ((pr - tr) ** 2).mean(), atol=1e-6)
    assert list(mt.keys()) == ["cls", "reg_MeanSquaredError", "reg_MeanAbsoluteError"]
    c = mt.clone(prefix="val_")
    assert list(c.keys(flatten=False)) == ["val_cls", "val_reg"]
    with pytest.raises(ValueError):
        mt.update({"cls": pc}, {"cls": tc})


def test_tracker():
    tr = tm.MetricTracker(tm.MeanSquaredError(), maximize=False)
    with pytest.raises(ValueError):
        tr.update(torch.randn(3), torch.randn(3))
    vals = []
    for _ in range(3):
        tr.increment()
        p, t = torch.randn(10), torch.randn(10)
        tr.update(p, t)
        vals.append(((p - t) ** 2).mean().item())
    all_ = tr.compute_all()
    np.testing.assert_allclose(all_.numpy(), vals, rtol=1e-5)
    best, step = tr.best_metric(return_step=True)
    assert step == int(np.argmin(vals)) and best == pytest.approx(min(vals), rel=1e-5)
    trc = tm.MetricTracker(tm.MetricCollection([tm.MeanSquaredError(), tm.MeanAbsoluteError()]), maximize=[False, False])
    trc.increment()
    trc.update(torch.randn(5), torch.randn(5))
    b = trc.best_metric()
    assert set(b) == {"MeanSquaredError", "MeanAbsoluteError"}


class _CountingNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.calls = 0
        self.num_features = 8
        self.lin = torch.nn.Linear(8, 8)

    def forward(self, x):
        self.calls += 1
        return self.lin(x.float())


def test_feature_share_runs_network_once():
    net = _CountingNet()
    fs = FeatureShare([FrechetInceptionDistance(feature=net), KernelInceptionDistance(feature=net, subset_size=4)])
    x = torch.randn(10, 8)
    fs.update(x, real=True)
    assert net.calls == 1


class _Extremes(tm.Metric):
    full_state_update = False

    def __init__(self):
        super().__init__()
        self.add_state("hi", torch.tensor(float("-inf")), dist_reduce_fx="max")
        self.add_state("lo", torch.tensor(float("inf")), dist_reduce_fx="min")

    def update(self, x):
        self.hi = torch.maximum(self.hi, x.max())
        self.lo = torch.minimum(self.lo, x.min())

    def compute(self):
        return torch.stack([self.lo, self.hi])


@pytest.mark.parametrize("make,arg_fn", [
    (lambda: tm.MeanSquaredError(), lambda g: (torch.randn(7, generator=g), torch.randn(7, generator=g))),
    (lambda: _Extremes(), lambda g: (torch.randn(7, generator=g),)),
    (lambda: tm.MeanMetric(), lambda g: (torch.randn(7, generator=g),)),
    (lambda: tm.CatMetric(), lambda g: (torch.randn(3, generator=g),)),
    (lambda: tm.MulticlassStatScores(4, average=None), lambda g: (torch.randint(0, 4, (9,), generator=g),
                                                                   torch.randint(0, 4, (9,), generator=g))),
])
@pytest.mark.parametrize("window", [1, 3])
def test_running_window_equals_metric_on_last_batches(make, arg_fn, window):
    """Running(window) == the wrapped metric fed only the last ``window`` batches (every reduction kind)."""
    g = torch.Generator().manual_seed(window)
    run = tm.wrappers.Running(make(), window=window)
    batches = []
    for _ in range(5):
        args = arg_fn(g)
        batches.append(args)
        run.update(*args)
        ref = make()
        for a in batches[-window:]:
            ref.update(*a)
        got, exp = run.compute(), ref.compute()
        if isinstance(ref, tm.CatMetric):  # the window is merged newest-first (as the reference's list merge)
            got, exp = got.sort().values, exp.sort().values
        torch.testing.assert_close(got, exp)
        run._computed = None


@pytest.mark.parametrize("shape,output_dim", [((50, 3), -1), ((50, 3, 4), 1), ((50, 4, 3), -1)])
@pytest.mark.parametrize("with_nans", [False, True])
def test_multioutput_nan_rows_match_per_output_filter(shape, output_dim, with_nans):
    g = torch.Generator().manual_seed(len(shape) + int(with_nans))
    p, t = torch.randn(*shape, generator=g), torch.randn(*shape, generator=g)
    if with_nans:
        p.view(-1)[torch.randperm(p.numel(), generator=g)[:9]] = float("nan")
        t.view(-1)[torch.randperm(t.numel(), generator=g)[:5]] = float("nan")
    m = tm.MultioutputWrapper(tm.MeanSquaredError(), num_outputs=3, output_dim=output_dim)
    m.update(p, t)
    got = m.compute()
    exp = []
    for i in range(3):
        pi, ti = p.narrow(output_dim, i, 1), t.narrow(output_dim, i, 1)
        bad = torch.isnan(pi.flatten(1)).any(1) | torch.isnan(ti.flatten(1)).any(1)
        exp.append(((pi[~bad] - ti[~bad]) ** 2).mean())
    torch.testing.assert_close(got, torch.stack(exp))
