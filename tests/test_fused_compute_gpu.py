"""Eager one-launch collection compute (``utils/fused_compute.py``): every value equals the CPU collection (the eager
per-member path), across repeated computes, reset, configuration changes, validation errors, device-side warnings,
copies of the collection, and results held across calls."""
import copy
import pickle
import warnings

import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import MetricCollection
from torchmetrics_amd import classification as C
from torchmetrics_amd import regression as R

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
NC = 10


def _cls():
    return MetricCollection({
        "acc": C.MulticlassAccuracy(NC, average="macro"), "prec": C.MulticlassPrecision(NC, average="macro"),
        "rec": C.MulticlassRecall(NC, average="macro"), "f1": C.MulticlassF1Score(NC, average="macro"),
        "fbeta": C.MulticlassFBetaScore(2.0, NC, average="macro"), "spec": C.MulticlassSpecificity(NC, average="macro"),
        "hamming": C.MulticlassHammingDistance(NC, average="macro"), "stat": C.MulticlassStatScores(NC, average="macro"),
        "jacc": C.MulticlassJaccardIndex(NC), "mcc": C.MulticlassMatthewsCorrCoef(NC), "kappa": C.MulticlassCohenKappa(NC),
        "cm": C.MulticlassConfusionMatrix(NC), "auroc": C.MulticlassAUROC(NC, thresholds=100),
        "ap": C.MulticlassAveragePrecision(NC, thresholds=100), "ece": C.MulticlassCalibrationError(NC, n_bins=15),
    }, compute_groups=True)


def _reg():
    return MetricCollection({"mse": R.MeanSquaredError(), "mae": R.MeanAbsoluteError(), "r2": R.R2Score(),
                             "pearson": R.PearsonCorrCoef(), "ev": R.ExplainedVariance()}, compute_groups=True)


def _batch(i, n=2048):
    g = torch.Generator().manual_seed(i)
    x = torch.randn(n, generator=g)
    return (torch.randn(n, NC, generator=g), torch.randint(0, NC, (n,), generator=g), x,
            x + 0.3 * torch.randn(n, generator=g))


def _check(a, b):
    assert set(a) == set(b)
    for k in b:
        torch.testing.assert_close(a[k].cpu(), b[k], atol=1e-5, rtol=1e-5, equal_nan=True, check_dtype=True)


def test_fused_compute_matches_cpu_collection():
    gc, gr, cc, cr = _cls().to(DEV), _reg().to(DEV), _cls(), _reg()
    held = None
    for i in range(5):
        p, t, x, y = _batch(i)
        gc.update(p.to(DEV), t.to(DEV))
        gr.update(x.to(DEV), y.to(DEV))
        cc.update(p, t)
        cr.update(x, y)
        a, b = gc.compute(), cc.compute()
        _check(a, b)
        _check(gr.compute(), cr.compute())
        if i == 2:
            held = {k: v.clone() for k, v in a.items()}
            held_live = a
    plan = gc.__dict__["_fused_plan"][1]
    assert plan.ok and {"acc", "prec", "f1", "jacc", "mcc", "kappa", "auroc", "ap"} <= plan.keys
    assert "ece" not in plan.keys  # list states stay eager
    assert gr.__dict__["_fused_plan"][1].keys >= {"mse", "mae", "r2"}
    for k in plan.keys:  # fused results handed out earlier are never overwritten by later computes
        assert torch.equal(held[k], held_live[k]), k


def test_reset_config_change_and_copies():
    gc, cc = _cls().to(DEV), _cls()
    for i in range(3):
        p, t, _, _ = _batch(10 + i)
        gc.update(p.to(DEV), t.to(DEV))
        cc.update(p, t)
        _check(gc.compute(), cc.compute())
    gc.reset()
    cc.reset()
    p, t, _, _ = _batch(20)
    gc.update(p.to(DEV), t.to(DEV))
    cc.update(p, t)
    _check(gc.compute(), cc.compute())
    for coll in (gc, cc):
        coll["acc"].average = "micro"
        coll["f1"].average = "weighted"
    _check(gc.compute(), cc.compute())
    gc.update(p.to(DEV), t.to(DEV))
    cc.update(p, t)
    _check(gc.compute(), cc.compute())
    for other in (copy.deepcopy(gc), pickle.loads(pickle.dumps(gc))):
        _check(other.compute(), cc.compute())
        other.update(p.to(DEV), t.to(DEV))
        _check(other.compute(), {k: v.cpu() for k, v in other.compute().items()})


def test_validation_error_and_device_warning_on_fused_path():
    gc = MetricCollection({"acc": C.MulticlassAccuracy(NC), "auroc": C.MulticlassAUROC(NC, thresholds=20)}).to(DEV)
    p, t, _, _ = _batch(30)
    for _ in range(2):
        gc.update(p.to(DEV), t.to(DEV))
        gc.compute()
    assert gc.__dict__["_fused_plan"][1].keys == {"acc", "auroc"}
    bad = t.clone()
    bad[0] = NC + 5
    gc.update(p.to(DEV), bad.to(DEV))
    with pytest.raises(RuntimeError, match="more unique values in `target`"):
        gc.compute()
    # a device-side warning of a fused member (Pearson's low-variance check, a flag the task kernel writes) joins the
    # collection's one status read and is emitted after the compute
    gr = MetricCollection({"mse": R.MeanSquaredError(), "pearson": R.PearsonCorrCoef()}).to(DEV)
    _, _, x, y = _batch(31)
    for _ in range(2):
        gr.update(x.to(DEV), y.to(DEV))
        gr.compute()
    assert gr.__dict__["_fused_plan"][1].keys == {"mse", "pearson"}
    gr.reset()
    gr.update(torch.full_like(x, 0.5).to(DEV), y.to(DEV))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        gr.compute()
    assert any("variance of predictions or target is close to zero" in str(x.message) for x in w)


def test_train_eval_toggle_keeps_fused_plan():
    """nn.Module.train() / eval() set ``training`` on every member: not a configuration change, so the recorded plan
    survives a train / validate loop (it used to be re-recorded at each switch and switched off after 8)."""
    gc, cc = _cls().to(DEV), _cls()
    plans = set()
    for i in range(12):
        p, t, _, _ = _batch(40 + i)
        gc.train() if i % 2 else gc.eval()
        gc.update(p.to(DEV), t.to(DEV))
        cc.update(p, t)
        _check(gc.compute(), cc.compute())
        if "_fused_plan" in gc.__dict__:
            plans.add(id(gc.__dict__["_fused_plan"][1]))
    assert len(plans) == 1
    assert not gc.__dict__.get("_fused_off")
    assert gc.__dict__.get("_fused_rebuilds", 0) == 1


def test_regression_collection_update_is_one_moments_pass(monkeypatch):
    """MSE / MAE / R2 / Pearson / EV on the same inputs: the plain sums read the unshifted twins (SP0 ...) of the
    centred sums the Pearson fold needs, so the whole collection update is ONE moments pass (one launch of the
    single-block kernel for an 8192-pair batch), and every value still equals the CPU collection."""
    from torchmetrics_amd import ops

    calls = []
    real = ops.moments_update

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)

    monkeypatch.setattr(ops, "moments_update", counting)
    gr, cr = _reg().to(DEV), _reg()
    for i in range(4):
        _, _, x, y = _batch(60 + i, n=8192)
        calls.clear()
        rp = gr.__dict__.get("_moments_replay")
        r0 = rp.calls if rp is not None else 0
        gr.update(x.to(DEV), y.to(DEV))
        # one moments call per step: merged through ops.moments_update, or the recorded call replayed
        rp = gr.__dict__.get("_moments_replay")
        n_gpu = len(calls) + ((rp.calls - r0) if rp is not None else 0)
        cr.update(x, y)  # (the CPU collection's own calls are not counted)
        if i > 0:  # (the first update finds the compute groups member by member)
            assert n_gpu == 1, n_gpu
        _check(gr.compute(), cr.compute())


def test_regression_collection_update_replay():
    """After one merged step the collection replays the recorded moments call (utils/fused_moments.py): the values
    still equal the CPU collection across steps, reset, a reconfigured member and a shape change (which fall back to
    the members' own updates and re-record)."""
    gr, cr = _reg().to(DEV), _reg()
    for i in range(7):  # (step 4 changes the batch size: step 5 re-records, step 6 replays)
        _, _, x, y = _batch(80 + i, n=4096 if i != 4 else 1000)
        gr.update(x.to(DEV), y.to(DEV))
        cr.update(x, y)
        _check(gr.compute(), cr.compute())
        if i == 2:
            rp = gr.__dict__.get("_moments_replay")
            assert rp is not None and rp.calls >= 1 and len(rp.members) == 5
            gr.reset()
            cr.reset()
    rp = gr.__dict__.get("_moments_replay")
    assert rp is not None and rp.calls >= 1
    # a bad shape still raises the member's error (the replay declines other shapes)
    with pytest.raises(RuntimeError):
        gr.update(torch.randn(10, device=DEV), torch.randn(11, device=DEV))


def test_dropped_results_reuse_the_output_buffer_held_ones_never_change():
    """A per-step compute() whose results were dropped reuses the plan's output buffer (no view construction); a kept
    result, a kept VIEW of a result and a member's cached compute() value each force a fresh buffer instead, so no
    handed-out tensor ever changes (utils/fused_compute.py CollectionPlan.run)."""
    gc, cc = _cls().to(DEV), _cls()
    ptrs = []
    kept, kept_view, snap, snap_view = None, None, None, None
    for i in range(8):
        p, t, _, _ = _batch(i)
        gc.update(p.to(DEV), t.to(DEV))
        cc.update(p, t)
        res = gc.compute()
        _check(res, cc.compute())
        ptrs.append(res["acc"].data_ptr())
        if i == 3:
            kept, snap = res["f1"], res["f1"].clone()
        if i == 5:
            kept_view, snap_view = res["mcc"].reshape(-1)[0:1], res["mcc"].reshape(-1)[0:1].clone()
        del res
    assert ptrs[2] == ptrs[1], "dropped results: the buffer is reused"
    assert ptrs[4] != ptrs[3], "a kept result forces a fresh buffer"
    assert ptrs[6] != ptrs[5], "a kept view of a result forces a fresh buffer"
    assert torch.equal(kept, snap) and torch.equal(kept_view, snap_view)
    # a second compute() without an update returns the members' cached values: the buffer holding them stays
    a = gc.compute()
    b = gc.compute()
    assert torch.equal(a["acc"], b["acc"])
