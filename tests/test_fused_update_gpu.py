"""Fused collection update (utils/fused_update.py, csrc/classification/family.hip): the few-class multiclass leaders
of a MetricCollection -- stat scores, confusion matrices, binned curves and calibration error -- updated by ONE rows
pass + one fold, against the same collection on the CPU (the per-member reference path): every compute value, the
states (list states included), probabilities vs logits (the batch-wide softmax decision), several dtypes and batch
sizes, compute groups on and off, and the deferred target-range error."""
import pytest
import torch

from torchmetrics_amd import MetricCollection
from torchmetrics_amd import classification as C

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
NC = 10


def _cls(compute_groups=True, nc=NC):
    return MetricCollection({
        "acc": C.MulticlassAccuracy(nc, average="macro"), "prec": C.MulticlassPrecision(nc, average="macro"),
        "f1": C.MulticlassF1Score(nc, average="weighted"), "micro": C.MulticlassAccuracy(nc, average="micro"),
        "stat": C.MulticlassStatScores(nc, average=None), "jacc": C.MulticlassJaccardIndex(nc),
        "mcc": C.MulticlassMatthewsCorrCoef(nc), "cm": C.MulticlassConfusionMatrix(nc),
        "auroc": C.MulticlassAUROC(nc, thresholds=100), "ap": C.MulticlassAveragePrecision(nc, thresholds=100),
        "ece": C.MulticlassCalibrationError(nc, n_bins=15),
    }, compute_groups=compute_groups)


def _check(a, b):
    assert set(a) == set(b)
    for k in b:
        torch.testing.assert_close(a[k].cpu(), b[k], atol=1e-5, rtol=1e-5, equal_nan=True, check_dtype=True, msg=k)


def _batch(i, n, nc=NC, probs=False, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(i)
    p = torch.randn(n, nc, generator=g)
    if probs:
        p = p.softmax(-1)
    return p.to(dtype), torch.randint(0, nc, (n,), generator=g)


def _plan(coll):
    entry = coll.__dict__.get("_family_plan")
    return None if entry is None else entry[1]


@pytest.mark.parametrize("compute_groups", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_fused_update_matches_cpu(compute_groups, dtype):
    g, c = _cls(compute_groups).to(DEV), _cls(compute_groups)
    for i, (n, probs) in enumerate([(2048, False), (777, True), (300_000, False), (8192, True), (1, False)]):
        p, t = _batch(i, n, probs=probs, dtype=dtype)
        g.update(p.to(DEV), t.to(DEV))
        c.update(p, t)
        _check(g.compute(), c.compute())
    plan = _plan(g)
    assert plan is not None and plan.ok and plan.calls >= 4
    # the list states of the calibration member hold the same elements as the per-member path (a softmax rounded to
    # 16 bits may land one ulp apart from the CPU's exp / sum order on rare elements)
    gc, cc = torch.cat(list(g["ece"].confidences)).cpu(), torch.cat(list(c["ece"].confidences))
    ulp = 0.0 if dtype == torch.float32 else 2.0 ** -8
    torch.testing.assert_close(gc, cc, atol=ulp + 1e-6, rtol=1e-6)
    if dtype != torch.float32:  # (fp32 softmax values differ from the CPU's in the last bits throughout)
        assert (gc != cc).float().mean() < 1e-4
    ga, ca = torch.cat(list(g["ece"].accuracies)).cpu(), torch.cat(list(c["ece"].accuracies))
    assert (ga != ca).float().mean() < 1e-4


def test_fused_update_states_equal_member_updates():
    """The fused path and the members' own (native) updates leave bit-identical integer states."""
    fused = _cls().to(DEV)
    solo = {k: m for k, m in _cls().to(DEV).items(keep_base=True)}
    for i in range(3):
        p, t = _batch(100 + i, 4096)
        fused.update(p.to(DEV), t.to(DEV))
        for m in solo.values():
            m.update(p.to(DEV), t.to(DEV))
    assert _plan(fused).calls >= 2
    for k in ("cm", "jacc", "mcc"):
        assert torch.equal(fused[k].confmat, solo[k].confmat), k
    for k in ("acc", "micro", "stat"):
        for s in ("tp", "fp", "tn", "fn"):
            assert torch.equal(getattr(fused[k], s), getattr(solo[k], s)), (k, s)
    assert torch.equal(fused["auroc"].confmat, solo["auroc"].confmat)


def test_fused_update_target_range_error_and_reset():
    g = _cls().to(DEV)
    p, t = _batch(5, 1024)
    g.update(p.to(DEV), t.to(DEV))
    g.update(p.to(DEV), t.to(DEV))
    g.update(p.to(DEV), torch.full((1024,), NC + 3, device=DEV))  # out of range: every member is flagged
    with pytest.raises(RuntimeError):
        g.compute()
    g.reset()
    g.update(p.to(DEV), t.to(DEV))
    c = _cls()
    c.update(p, t)
    _check(g.compute(), c.compute())


def test_fused_update_falls_back_off_path():
    """kwargs, CPU inputs or a different class count go through the members' own updates (same results)."""
    g, c = _cls().to(DEV), _cls()
    p, t = _batch(9, 512)
    g.update(preds=p.to(DEV), target=t.to(DEV))
    c.update(preds=p, target=t)
    g.update(p.to(DEV), t.to(DEV))
    c.update(p, t)
    _check(g.compute(), c.compute())


@pytest.mark.parametrize("nc", [2, 3, 5, 8, 13, 16, 17, 33])
@pytest.mark.parametrize("nan_rows", [False, True])
def test_fused_update_group_widths(nc, nan_rows):
    """family_rows_g_kernel's group exchanges: DPP butterflies / row broadcasts for G <= 16 lanes per row (G = 2, 4,
    8, 16), ds_bpermute shuffles above (32, 64) -- every class count against the CPU collection, with NaN rows (the
    NaN-ignoring max differs from the argmax max there)."""
    g, c = _cls(nc=nc).to(DEV), _cls(nc=nc)
    for i, n in enumerate([4096, 333]):
        p, t = _batch(40 + i, n, nc=nc)
        if nan_rows:
            p[::97, nc // 2] = float("nan")
        g.update(p.to(DEV), t.to(DEV))
        c.update(p, t)
    _check(g.compute(), c.compute())
    assert _plan(g) is not None and _plan(g).calls >= 1


@pytest.mark.parametrize("n_bins", [15, 40])
def test_calibration_error_nan_rows_standalone(n_bins):
    """NaN confidences land in the last bin, where torch.bucketize(right=True) puts them in the reference
    (calib_bins_private_kernel for <= 16 bounds, calib_bins_kernel above)."""
    g_m, c_m = C.MulticlassCalibrationError(5, n_bins=n_bins).to(DEV), C.MulticlassCalibrationError(5, n_bins=n_bins)
    for i in range(2):
        p, t = _batch(70 + i, 2000, nc=5)
        p[::13, 2] = float("nan")
        g_m.update(p.to(DEV), t.to(DEV))
        c_m.update(p, t)
    torch.testing.assert_close(g_m.compute().cpu(), c_m.compute(), atol=1e-5, rtol=1e-5, equal_nan=True)
