"""Curve family (PR curve, ROC, AUROC, AP, operating points) vs scikit-learn / direct numpy oracles.

The binned path is checked against a direct ``preds[:, None] >= thresholds`` numpy count (the reference definition,
``F/classification/precision_recall_curve.py:210-250``); the GPU kernel is checked against the CPU implementation
for every mode / dtype / ignore_index / threshold layout.
"""
from functools import partial

import numpy as np
import pytest
import torch
from sklearn import metrics as skm

import torchmetrics_amd as tm
import torchmetrics_amd.functional as F
from torchmetrics_amd import ops
from tests.helpers import assert_close, run_class_test, run_ddp_class_test, run_functional_test

NB, BS, C, L = 4, 64, 5, 3
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _np(x):
    return x.detach().cpu().numpy()


def _sigmoid_if_needed(p):
    return p if ((p >= 0) & (p <= 1)).all() else 1 / (1 + np.exp(-p))


def _softmax_if_needed(p):
    if ((p >= 0) & (p <= 1)).all():
        return p
    e = np.exp(p - p.max(1, keepdims=True))
    return e / e.sum(1, keepdims=True)


def _binary(kind, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 2, (NB, BS), generator=g)
    p = torch.rand(NB, BS, generator=g) if kind == "prob" else torch.randn(NB, BS, generator=g) * 3
    return p, t


def _multiclass(kind, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, C, (NB, BS), generator=g)
    p = torch.randn(NB, BS, C, generator=g)
    return (p.softmax(-1) if kind == "prob" else p * 2), t


def _multilabel(kind, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 2, (NB, BS, L), generator=g)
    p = torch.rand(NB, BS, L, generator=g) if kind == "prob" else torch.randn(NB, BS, L, generator=g) * 3
    return p, t


# --------------------------------------------------------------------------------------------- oracles
def _sk_binary_auroc(p, t, ignore_index=None):
    p, t = _np(p).ravel(), _np(t).ravel()
    if ignore_index is not None:
        p, t = p[t != ignore_index], t[t != ignore_index]
    return skm.roc_auc_score(t, _sigmoid_if_needed(p))


def _sk_binary_ap(p, t, ignore_index=None):
    p, t = _np(p).ravel(), _np(t).ravel()
    if ignore_index is not None:
        p, t = p[t != ignore_index], t[t != ignore_index]
    return skm.average_precision_score(t, _sigmoid_if_needed(p))


def _np_binned_confmat(p, t, thr):
    pred = p[:, None] >= thr[None, :]
    pos = (t == 1)[:, None]
    return np.stack([(~pred & ~pos).sum(0), (pred & ~pos).sum(0), (~pred & pos).sum(0), (pred & pos).sum(0)], -1)


def _binned_binary_auroc(p, t, n_thr):
    p, t = _sigmoid_if_needed(_np(p).ravel()), _np(t).ravel()
    thr = np.linspace(0, 1, n_thr, dtype=np.float32)
    cm = _np_binned_confmat(p, t, thr)
    tn, fp, fn, tp = cm.T.astype(np.float64)
    tpr = np.where(tp + fn > 0, tp / np.maximum(tp + fn, 1), 0)[::-1]
    fpr = np.where(fp + tn > 0, fp / np.maximum(fp + tn, 1), 0)[::-1]
    return np.trapz(tpr, fpr)


def _binned_binary_ap(p, t, n_thr):
    p, t = _sigmoid_if_needed(_np(p).ravel()), _np(t).ravel()
    thr = np.linspace(0, 1, n_thr, dtype=np.float32)
    tn, fp, fn, tp = _np_binned_confmat(p, t, thr).T.astype(np.float64)
    prec = np.concatenate([np.where(tp + fp > 0, tp / np.maximum(tp + fp, 1), 0), [1.0]])
    rec = np.concatenate([np.where(tp + fn > 0, tp / np.maximum(tp + fn, 1), 0), [0.0]])
    return -np.sum((rec[1:] - rec[:-1]) * prec[:-1])


def _sk_multiclass(fn, p, t, average, ignore_index=None):
    p, t = _np(p).reshape(-1, C), _np(t).ravel()
    if ignore_index is not None:
        p, t = p[t != ignore_index], t[t != ignore_index]
    p = _softmax_if_needed(p)
    res = []
    for i in range(C):
        pos = t == i
        if pos.all() or not pos.any():  # reference: AUROC 0 (zero tpr/fpr), AP nan (0/0 recall)
            res.append(0.0 if fn is skm.roc_auc_score else np.nan)
        else:
            res.append(fn(pos, p[:, i]))
    res = np.array(res)
    if average in (None, "none"):
        return res
    ok = ~np.isnan(res)
    if average == "macro":
        return res[ok].mean()
    w = np.bincount(t, minlength=C)[ok]
    return (res[ok] * w / w.sum()).sum()


def _sk_multilabel(fn, p, t, average, ignore_index=None):
    p, t = _np(p).reshape(-1, L), _np(t).reshape(-1, L)
    p = _sigmoid_if_needed(p)
    if average == "micro":
        pf, tf = p.ravel(), t.ravel()
        keep = tf != ignore_index if ignore_index is not None else np.ones_like(tf, dtype=bool)
        return fn(tf[keep], pf[keep])
    res = []
    for i in range(L):
        keep = t[:, i] != ignore_index if ignore_index is not None else np.ones(len(t), dtype=bool)
        res.append(fn(t[keep, i], p[keep, i]))
    res = np.array(res)
    if average in (None, "none"):
        return res
    if average == "macro":
        return res.mean()
    w = (t == 1).sum(0)
    return (res * w / w.sum()).sum()


# ------------------------------------------------------------------------------------------------ binary
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit"])
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_binary_auroc_ap_unbinned(device, kind, ignore_index):
    p, t = _binary(kind)
    if ignore_index is not None:
        t[:, ::7] = ignore_index
    run_functional_test(p, t, F.binary_auroc, partial(_sk_binary_auroc, ignore_index=ignore_index),
                        {"ignore_index": ignore_index}, atol=1e-5, device=device)
    run_class_test(p, t, tm.BinaryAUROC, partial(_sk_binary_auroc, ignore_index=ignore_index),
                   {"ignore_index": ignore_index}, atol=1e-5, device=device)
    run_class_test(p, t, tm.BinaryAveragePrecision, partial(_sk_binary_ap, ignore_index=ignore_index),
                   {"ignore_index": ignore_index}, atol=1e-5, device=device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit"])
@pytest.mark.parametrize("n_thr", [5, 100])
def test_binary_auroc_ap_binned(device, kind, n_thr):
    p, t = _binary(kind, seed=1)
    run_class_test(p, t, tm.BinaryAUROC, partial(_binned_binary_auroc, n_thr=n_thr), {"thresholds": n_thr},
                   atol=1e-5, device=device)
    run_class_test(p, t, tm.BinaryAveragePrecision, partial(_binned_binary_ap, n_thr=n_thr), {"thresholds": n_thr},
                   atol=1e-5, device=device)


@pytest.mark.parametrize("device", DEVICES)
def test_binary_pr_curve_and_roc_vs_sklearn(device):
    p, t = _binary("prob", seed=3)
    p = (p * 20).round() / 20  # ties
    for i in range(NB):
        prec, rec, thr = F.binary_precision_recall_curve(p[i].to(device), t[i].to(device))
        sp, sr, st = skm.precision_recall_curve(_np(t[i]), _np(p[i]))
        assert_close(prec, sp, atol=1e-6)
        assert_close(rec, sr, atol=1e-6)
        assert_close(thr, st, atol=1e-6)
        fpr, tpr, thr = F.binary_roc(p[i].to(device), t[i].to(device))
        sf, stp, _ = skm.roc_curve(_np(t[i]), _np(p[i]), drop_intermediate=False)
        assert_close(fpr, sf, atol=1e-6)
        assert_close(tpr, stp, atol=1e-6)


def test_binary_binned_matches_reference_confmat_layout():
    p, t = _binary("prob", seed=4)
    thr = torch.tensor([0.9, 0.1, 0.5, 0.3])  # unsorted user thresholds keep their order
    m = tm.BinaryPrecisionRecallCurve(thresholds=thr)
    m.update(p[0], t[0])
    ref = _np_binned_confmat(_np(p[0]), _np(t[0]), _np(thr)).reshape(-1, 2, 2)
    np.testing.assert_array_equal(_np(m.confmat), ref)


def test_binary_max_fpr():
    p, t = _binary("prob", seed=5)
    ours = F.binary_auroc(p.flatten(), t.flatten(), max_fpr=0.3)
    ref = skm.roc_auc_score(_np(t).ravel(), _np(p).ravel(), max_fpr=0.3)
    assert_close(ours, ref, atol=1e-5)


# -------------------------------------------------------------------------------------------- multiclass
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit"])
@pytest.mark.parametrize("average", ["macro", "weighted", "none"])
@pytest.mark.parametrize("ignore_index", [None, 1])
def test_multiclass_auroc_ap_unbinned(device, kind, average, ignore_index):
    p, t = _multiclass(kind)
    args = {"num_classes": C, "average": average, "ignore_index": ignore_index}
    run_class_test(p, t, tm.MulticlassAUROC,
                   partial(_sk_multiclass, skm.roc_auc_score, average=average, ignore_index=ignore_index), args,
                   atol=1e-5, device=device, check_batch=ignore_index is None)
    run_class_test(p, t, tm.MulticlassAveragePrecision,
                   partial(_sk_multiclass, skm.average_precision_score, average=average, ignore_index=ignore_index),
                   args, atol=1e-5, device=device, check_batch=ignore_index is None)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit"])
def test_multiclass_binned_vs_numpy(device, kind):
    p, t = _multiclass(kind, seed=2)
    thr = torch.linspace(0, 1, 17)
    m = tm.MulticlassPrecisionRecallCurve(num_classes=C, thresholds=17).to(device)
    for i in range(NB):
        m.update(p[i].to(device), t[i].to(device))
    pp = _softmax_if_needed(_np(p).reshape(-1, C).astype(np.float64))
    tt = _np(t).ravel()
    ref = np.stack([_np_binned_confmat(pp[:, c], (tt == c).astype(np.int64), _np(thr)) for c in range(C)], 1)
    # per-batch softmax decision is identical here (all batches are logits or all probs)
    np.testing.assert_array_equal(_np(m.confmat).reshape(17, C, 4), ref)
    prec, rec, _ = m.compute()
    assert prec.shape == (C, 18) and rec.shape == (C, 18)


@pytest.mark.parametrize("device", DEVICES)
def test_multiclass_micro_curve(device):
    p, t = _multiclass("prob", seed=6)
    pm = tm.MulticlassPrecisionRecallCurve(num_classes=C, thresholds=11, average="micro").to(device)
    pm.update(p[0].to(device), t[0].to(device))
    onehot = torch.nn.functional.one_hot(t[0], C).flatten()
    prec, rec, _ = F.binary_precision_recall_curve(p[0].flatten(), onehot, thresholds=11)
    mp, mr, _ = pm.compute()
    assert_close(mp, prec)
    assert_close(mr, rec)


# -------------------------------------------------------------------------------------------- multilabel
@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit"])
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", "none"])
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_multilabel_auroc_ap_unbinned(device, kind, average, ignore_index):
    p, t = _multilabel(kind)
    if ignore_index is not None:
        t[:, ::5, 0] = ignore_index
    args = {"num_labels": L, "average": average, "ignore_index": ignore_index}
    run_class_test(p, t, tm.MultilabelAUROC,
                   partial(_sk_multilabel, skm.roc_auc_score, average=average, ignore_index=ignore_index), args,
                   atol=1e-5, device=device)
    run_class_test(p, t, tm.MultilabelAveragePrecision,
                   partial(_sk_multilabel, skm.average_precision_score, average=average, ignore_index=ignore_index),
                   args, atol=1e-5, device=device)


@pytest.mark.parametrize("device", DEVICES)
def test_multilabel_binned_ignore(device):
    p, t = _multilabel("logit", seed=7)
    t[:, ::3, 1] = -1
    m = tm.MultilabelROC(num_labels=L, thresholds=9, ignore_index=-1).to(device)
    for i in range(NB):
        m.update(p[i].to(device), t[i].to(device))
    pp = _sigmoid_if_needed(_np(p).reshape(-1, L))  # every batch holds logits
    tt = _np(t).reshape(-1, L)
    thr = np.linspace(0, 1, 9, dtype=np.float32)
    for j in range(L):
        keep = tt[:, j] != -1
        ref = _np_binned_confmat(pp[keep, j], tt[keep, j], thr)
        np.testing.assert_array_equal(_np(m.confmat[:, j]).reshape(9, 4), ref)


# ---------------------------------------------------------------------------------------- operating points
@pytest.mark.parametrize("device", DEVICES)
def test_recall_at_fixed_precision_vs_sklearn(device):
    p, t = _binary("prob", seed=8)
    for i in range(NB):
        r, thr = F.binary_recall_at_fixed_precision(p[i].to(device), t[i].to(device), min_precision=0.55)
        sp, sr, st = skm.precision_recall_curve(_np(t[i]), _np(p[i]))
        ok = sp[:-1] >= 0.55
        assert_close(r, sr[:-1][ok].max() if ok.any() else 0.0, atol=1e-6)
    m = tm.MulticlassSpecificityAtSensitivity(num_classes=C, min_sensitivity=0.5, thresholds=None).to(device)
    pc, tc = _multiclass("prob", seed=9)
    m.update(pc[0].to(device), tc[0].to(device))
    spec, thr = m.compute()
    assert spec.shape == (C,) and thr.shape == (C,)
    w = tm.SensitivityAtSpecificity(task="multilabel", num_labels=L, min_specificity=0.5, thresholds=20)
    pl, tl = _multilabel("prob", seed=10)
    w.update(pl[0], tl[0])
    sens, _ = w.compute()
    assert sens.shape == (L,)
    bp = tm.PrecisionAtFixedRecall(task="binary", min_recall=0.5)
    bp.update(p[0], t[0])
    prec, _ = bp.compute()
    sp, sr, _ = skm.precision_recall_curve(_np(t[0]), _np(p[0]))
    assert_close(prec, sp[sr >= 0.5].max(), atol=1e-6)


# --------------------------------------------------------------------------------------------------- DDP
@pytest.mark.ddp
@pytest.mark.parametrize("thresholds", [None, 50])
def test_binary_auroc_ddp(thresholds):
    p, t = _binary("prob", seed=11)
    ref = _sk_binary_auroc if thresholds is None else partial(_binned_binary_auroc, n_thr=thresholds)
    run_ddp_class_test(p, t, tm.BinaryAUROC, ref, {"thresholds": thresholds}, atol=1e-5)


# ---------------------------------------------------------------------------------------------- kernel parity
@pytest.mark.gpu
@pytest.mark.parametrize("mode", [ops.CURVE_BINARY, ops.CURVE_MULTILABEL, ops.CURVE_MULTICLASS])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
@pytest.mark.parametrize("n_thr", [1, 7, 100, 5000])
@pytest.mark.parametrize("logits", [False, True])
@pytest.mark.parametrize("ignore", [False, True])
def test_curve_kernel_matches_cpu(mode, dtype, n_thr, logits, ignore):
    g = torch.Generator().manual_seed(n_thr)
    n, k = 3001, (1 if mode == ops.CURVE_BINARY else 130)
    if mode == ops.CURVE_MULTICLASS:
        p = torch.randn(n, k, generator=g)
        p = p * 3 if logits else p.softmax(-1)
        t = torch.randint(0, k, (n,), generator=g)
        if ignore:
            t[::9] = -100
    else:
        shape = (n,) if mode == ops.CURVE_BINARY else (n, k)
        p = torch.randn(shape, generator=g) * 3 if logits else torch.rand(shape, generator=g)
        t = torch.randint(0, 2, shape, generator=g)
        if ignore:
            t.view(-1)[::9] = -100
    p = p.to(dtype)
    thr = torch.rand(n_thr, generator=g) if n_thr != 100 else torch.linspace(0, 1, n_thr)
    ts, perm = thr.double().sort()
    hcols = 1 if mode == ops.CURVE_BINARY else k
    shape = (n_thr, 2, 2) if hcols == 1 else (n_thr, hcols, 2, 2)
    ii = -100 if ignore else None
    cpu = torch.zeros(shape, dtype=torch.long)
    ops.curve_update(p, t, ts, perm, None, None, cpu, torch.zeros(1, dtype=torch.int32), mode, ii)
    dev = torch.device("cuda")
    gpu = torch.zeros(shape, dtype=torch.long, device=dev)
    hist = torch.zeros((n_thr + 1) * hcols * 2, dtype=torch.int32, device=dev)
    ctl = torch.zeros(1, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(2):  # the workspace must come back zeroed
        ops.curve_update(p.to(dev), t.to(dev), ts.to(dev), perm.to(dev), hist, ctl, gpu, err, mode, ii)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert int(hist.abs().sum().item()) == 0 and int(ctl.item()) == 0
    # float16/bfloat16 softmax / sigmoid may differ by one ulp from ATen right at a threshold: allow a tiny slack
    diff = (gpu.cpu() - 2 * cpu).abs().max().item()
    tol = 0 if (dtype in (torch.float32, torch.float64) and not logits) else 6
    assert diff <= tol, diff


@pytest.mark.gpu
def test_curve_kernel_flags_bad_targets():
    dev = torch.device("cuda")
    m = tm.BinaryAUROC(thresholds=10).to(dev)
    m.update(torch.rand(10, device=dev), torch.tensor([0, 1, 2, 0, 1, 0, 1, 0, 1, 0], device=dev))
    with pytest.raises(RuntimeError):
        m.compute()
