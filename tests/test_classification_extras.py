"""Calibration error, hinge, label ranking, exact match, group fairness and Dice vs sklearn / numpy oracles."""
from functools import partial

import numpy as np
import pytest
import torch
from sklearn import metrics as skm

import torchmetrics_amd as tm
import torchmetrics_amd.functional as F
from tests.helpers import assert_close, run_class_test, run_ddp_class_test, run_functional_test

NB, BS, C, L = 4, 64, 5, 4
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _np(x):
    return x.detach().cpu().numpy()


def _sig(p):
    return p if ((p >= 0) & (p <= 1)).all() else 1 / (1 + np.exp(-p))


def _soft(p):
    if ((p >= 0) & (p <= 1)).all():
        return p
    e = np.exp(p - p.max(1, keepdims=True))
    return e / e.sum(1, keepdims=True)


# ------------------------------------------------------------------------------------------- calibration error
def _np_ce(conf, acc, n_bins, norm):
    bounds = np.linspace(0, 1, n_bins + 1)
    idx = np.clip(np.searchsorted(bounds, conf, side="right") - 1, 0, n_bins)
    cnt = np.bincount(idx, minlength=n_bins + 1).astype(np.float64)
    cs = np.bincount(idx, weights=conf, minlength=n_bins + 1)
    ac = np.bincount(idx, weights=acc, minlength=n_bins + 1)
    with np.errstate(invalid="ignore", divide="ignore"):
        cb, ab = np.nan_to_num(cs / cnt), np.nan_to_num(ac / cnt)
    prop = cnt / cnt.sum()
    if norm == "l1":
        return np.sum(np.abs(ab - cb) * prop)
    if norm == "max":
        return np.max(np.abs(ab - cb))
    return np.sqrt(np.sum((ab - cb) ** 2 * prop))


def _bin_ce_ref(p, t, n_bins, norm):
    return _np_ce(_sig(_np(p).ravel().astype(np.float64)), _np(t).ravel().astype(np.float64), n_bins, norm)


def _mc_ce_ref(p, t, n_bins, norm):
    pp = _soft(_np(p).reshape(-1, C).astype(np.float64))
    conf, pred = pp.max(1), pp.argmax(1)
    return _np_ce(conf, (pred == _np(t).ravel()).astype(np.float64), n_bins, norm)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("norm", ["l1", "l2", "max"])
@pytest.mark.parametrize("kind", ["prob", "logit"])
def test_calibration_error(device, norm, kind):
    g = torch.Generator().manual_seed(0)
    p = torch.rand(NB, BS, generator=g) if kind == "prob" else torch.randn(NB, BS, generator=g) * 2
    t = torch.randint(0, 2, (NB, BS), generator=g)
    run_class_test(p, t, tm.BinaryCalibrationError, partial(_bin_ce_ref, n_bins=10, norm=norm),
                   {"n_bins": 10, "norm": norm}, atol=1e-5, device=device)
    pm = torch.randn(NB, BS, C, generator=g)
    pm = pm.softmax(-1) if kind == "prob" else pm
    tmc = torch.randint(0, C, (NB, BS), generator=g)
    run_class_test(pm, tmc, tm.MulticlassCalibrationError, partial(_mc_ce_ref, n_bins=10, norm=norm),
                   {"num_classes": C, "n_bins": 10, "norm": norm}, atol=1e-5, device=device)


# ---------------------------------------------------------------------------------------------------- hinge
def _bin_hinge_ref(p, t, squared):
    p, t = _sig(_np(p).ravel().astype(np.float64)), _np(t).ravel()
    m = np.clip(1 - np.where(t == 1, p, -p), 0, None)
    return (m**2 if squared else m).mean()


def _mc_hinge_ref(p, t, squared, mode):
    p, t = _soft(_np(p).reshape(-1, C).astype(np.float64)), _np(t).ravel()
    oh = np.eye(C, dtype=bool)[t]
    if mode == "crammer-singer":
        margin = p[oh] - np.where(oh, -np.inf, p).max(1)
    else:
        margin = np.where(oh, p, -p)
    m = np.clip(1 - margin, 0, None)
    m = m**2 if squared else m
    return m.sum(0) / len(t)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("squared", [False, True])
@pytest.mark.parametrize("mode", ["crammer-singer", "one-vs-all"])
def test_hinge(device, squared, mode):
    g = torch.Generator().manual_seed(1)
    p, t = torch.randn(NB, BS, generator=g), torch.randint(0, 2, (NB, BS), generator=g)
    run_class_test(p, t, tm.BinaryHingeLoss, partial(_bin_hinge_ref, squared=squared), {"squared": squared},
                   atol=1e-5, device=device)
    pm, tmc = torch.randn(NB, BS, C, generator=g), torch.randint(0, C, (NB, BS), generator=g)
    run_class_test(pm, tmc, tm.MulticlassHingeLoss, partial(_mc_hinge_ref, squared=squared, mode=mode),
                   {"num_classes": C, "squared": squared, "multiclass_mode": mode}, atol=1e-5, device=device)


def test_hinge_ignore_index():
    p, t = torch.randn(40), torch.randint(0, 2, (40,))
    t[::4] = -1
    keep = t != -1
    assert_close(F.binary_hinge_loss(p, t, ignore_index=-1), _bin_hinge_ref(p[keep], t[keep], False), atol=1e-6)


# -------------------------------------------------------------------------------------------------- ranking
def _sk_rank(fn, p, t):
    return fn(_np(t), _sig(_np(p)))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize(
    "cls, sk",
    [
        (tm.MultilabelCoverageError, skm.coverage_error),
        (tm.MultilabelRankingAveragePrecision, skm.label_ranking_average_precision_score),
        (tm.MultilabelRankingLoss, skm.label_ranking_loss),
    ],
)
def test_ranking(device, cls, sk):
    g = torch.Generator().manual_seed(2)
    p = torch.rand(NB, BS, L, generator=g)
    if cls is not tm.MultilabelRankingLoss:  # the ranking loss breaks ties by argsort order (as the reference)
        p[:, :8] = (p[:, :8] * 3).round() / 3
    t = torch.randint(0, 2, (NB, BS, L), generator=g)
    run_class_test(p, t, cls, partial(_sk_rank, sk), {"num_labels": L}, atol=1e-5, device=device)


# ---------------------------------------------------------------------------------------------- exact match
@pytest.mark.parametrize("device", DEVICES)
def test_exact_match(device):
    g = torch.Generator().manual_seed(3)
    p = torch.randint(0, 3, (NB, BS, 6), generator=g)
    t = p.clone()
    t[:, ::3, 2] = (t[:, ::3, 2] + 1) % 3

    def ref(pp, tt):
        return (_np(pp).reshape(len(pp), -1) == _np(tt).reshape(len(tt), -1)).all(1).mean()

    run_class_test(p, t, tm.MulticlassExactMatch, ref, {"num_classes": 3}, device=device)
    pl = torch.rand(NB, BS, L, generator=g)
    tl = (pl > 0.5).long()
    tl[:, ::5, 1] = 1 - tl[:, ::5, 1]
    run_class_test(pl, tl, tm.MultilabelExactMatch,
                   lambda a, b: ((_np(a) > 0.5) == _np(b)).all(-1).mean(), {"num_labels": L}, device=device)


@pytest.mark.parametrize("ignore_index", [0, -1])
@pytest.mark.parametrize("samplewise", [False, True])
def test_multilabel_exact_match_ignore_index(ignore_index, samplewise):
    """Reference baseline ``_baseline_exact_match_multilabel`` (T/classification/test_exact_match.py:150-171): an
    ignored target becomes -1 while the prediction stays 0/1, so a sample with an ignored position never matches."""
    from torchmetrics_amd.functional.classification import multilabel_exact_match

    g = torch.Generator().manual_seed(11)
    preds = torch.rand(64, L, 3, generator=g)
    target = (preds > 0.5).long()
    target[::7, 1, 0] = 1 - target[::7, 1, 0]
    if ignore_index == -1:
        target[::3, 2, 1] = -1
    p_np, t_np = (_np(preds) > 0.5).astype(np.int64), _np(target).astype(np.int64).copy()
    t_np[t_np == ignore_index] = -1
    if samplewise:
        exp = ((p_np == t_np).sum(1) == L).sum(1) / p_np.shape[2]
    else:
        pp, tt = np.moveaxis(p_np, 1, -1).reshape(-1, L), np.moveaxis(t_np, 1, -1).reshape(-1, L)
        exp = ((pp == tt).sum(1) == L).mean()
    avg = "samplewise" if samplewise else "global"
    got = multilabel_exact_match(preds, target, L, multidim_average=avg, ignore_index=ignore_index)
    np.testing.assert_allclose(_np(got), exp, rtol=1e-6)


# -------------------------------------------------------------------------------------------- group fairness
@pytest.mark.parametrize("device", DEVICES)
def test_group_fairness(device):
    g = torch.Generator().manual_seed(4)
    p, t = torch.rand(200, generator=g), torch.randint(0, 2, (200,), generator=g)
    groups = torch.randint(0, 3, (200,), generator=g)
    m = tm.BinaryFairness(num_groups=3).to(device)
    m.update(p.to(device), t.to(device), groups.to(device))
    res = m.compute()
    pred = _np(p) > 0.5
    tt, gg = _np(t), _np(groups)
    pos_rate = np.array([pred[gg == k].mean() for k in range(3)])
    tpr = np.array([(pred & (tt == 1))[gg == k].sum() / (tt[gg == k] == 1).sum() for k in range(3)])
    dp_key = [k for k in res if k.startswith("DP")][0]
    eo_key = [k for k in res if k.startswith("EO")][0]
    assert dp_key == f"DP_{pos_rate.argmin()}_{pos_rate.argmax()}"
    assert_close(res[dp_key], pos_rate.min() / pos_rate.max(), atol=1e-6)
    assert_close(res[eo_key], tpr.min() / tpr.max(), atol=1e-6)
    rates = F.binary_groups_stat_rates(p, t, groups, 3)
    assert set(rates) == {"group_0", "group_1", "group_2"}
    gsr = tm.BinaryGroupStatRates(num_groups=3)
    gsr.update(p, t, groups)
    assert_close(gsr.compute()["group_1"], rates["group_1"])


# ---------------------------------------------------------------------------------------------------- dice
def _np_dice_micro(p, t):
    pp, tt = _np(p).ravel() >= 0.5, _np(t).ravel() == 1
    tp, fp, fn = (pp & tt).sum(), (pp & ~tt).sum(), (~pp & tt).sum()
    return 2 * tp / (2 * tp + fp + fn)


def test_dice():
    g = torch.Generator().manual_seed(5)
    p, t = torch.rand(NB, BS, generator=g), torch.randint(0, 2, (NB, BS), generator=g)
    run_class_test(p, t, tm.Dice, _np_dice_micro, {}, atol=1e-6)
    pm, tmc = torch.randn(BS, C, generator=g).softmax(-1), torch.randint(0, C, (BS,), generator=g)
    ours = F.dice(pm, tmc, average="macro", num_classes=C)
    pred = _np(pm).argmax(1)
    tt = _np(tmc)
    scores = [2 * ((pred == c) & (tt == c)).sum() / ((pred == c).sum() + (tt == c).sum()) for c in range(C)]
    assert_close(ours, np.mean(scores), atol=1e-6)
    assert_close(F.dice(pm, tmc, average="none", num_classes=C), scores, atol=1e-6)


@pytest.mark.ddp
def test_hinge_ddp():
    g = torch.Generator().manual_seed(6)
    p, t = torch.randn(NB, BS, generator=g), torch.randint(0, 2, (NB, BS), generator=g)
    run_ddp_class_test(p, t, tm.BinaryHingeLoss, partial(_bin_hinge_ref, squared=False), {}, atol=1e-5)
