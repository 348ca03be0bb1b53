"""Stat-score family + confusion-matrix family vs scikit-learn oracles (reference test model: ``T/classification``).

Each case runs the functional and the module API on CPU, and on the GPU (``gpu`` marker) through the HIP kernels.
"""
from functools import partial

import numpy as np
import pytest
import torch
from sklearn import metrics as skm

import torchmetrics_amd as tm
import torchmetrics_amd.functional as F
from tests.helpers import assert_close, run_class_test, run_ddp_class_test, run_functional_test

NB, BS, C, L = 4, 32, 5, 4

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _np(x):
    return x.detach().cpu().numpy()


# ------------------------------------------------------------------------------------------------------- inputs
def _binary_inputs(kind):
    t = torch.randint(0, 2, (NB, BS))
    if kind == "prob":
        p = torch.rand(NB, BS)
    elif kind == "logit":
        p = torch.randn(NB, BS) * 3
    else:
        p = torch.randint(0, 2, (NB, BS))
    return p, t


def _multiclass_inputs(kind):
    t = torch.randint(0, C, (NB, BS))
    if kind == "prob":
        p = torch.randn(NB, BS, C).softmax(-1)
    elif kind == "logit":
        p = torch.randn(NB, BS, C)
    else:
        p = torch.randint(0, C, (NB, BS))
    return p, t


def _multilabel_inputs(kind):
    t = torch.randint(0, 2, (NB, BS, L))
    if kind == "prob":
        p = torch.rand(NB, BS, L)
    elif kind == "logit":
        p = torch.randn(NB, BS, L) * 3
    else:
        p = torch.randint(0, 2, (NB, BS, L))
    return p, t


# ------------------------------------------------------------------------------------------------------ oracles
def _binary_labels(p, t, ignore_index):
    p, t = p.flatten(), t.flatten()
    if p.is_floating_point():
        if not ((p >= 0) & (p <= 1)).all():
            p = p.sigmoid()
        p = (p > 0.5).long()
    keep = t != ignore_index if ignore_index is not None else torch.ones_like(t, dtype=torch.bool)
    return _np(p[keep]), _np(t[keep])


def _ref_binary(kind, p, t, ignore_index=None):
    pp, tt = _binary_labels(p, t, ignore_index)
    if kind == "accuracy":
        return skm.accuracy_score(tt, pp)
    if kind == "precision":
        return skm.precision_score(tt, pp, zero_division=0)
    if kind == "recall":
        return skm.recall_score(tt, pp, zero_division=0)
    if kind == "f1":
        return skm.f1_score(tt, pp, zero_division=0)
    if kind == "fbeta2":
        return skm.fbeta_score(tt, pp, beta=2.0, zero_division=0)
    if kind == "hamming":
        return 1 - skm.accuracy_score(tt, pp)
    if kind == "specificity":
        tn, fp, _, _ = skm.confusion_matrix(tt, pp, labels=[0, 1]).ravel()
        return tn / (tn + fp) if tn + fp else 0.0
    if kind == "confmat":
        return skm.confusion_matrix(tt, pp, labels=[0, 1])
    if kind == "kappa":
        return skm.cohen_kappa_score(tt, pp)
    if kind == "jaccard":
        return skm.jaccard_score(tt, pp, zero_division=0)
    if kind == "mcc":
        return skm.matthews_corrcoef(tt, pp)
    raise ValueError(kind)


def _mc_labels(p, t, ignore_index):
    if p.is_floating_point():
        p = p.argmax(-1)
    p, t = p.flatten(), t.flatten()
    keep = t != ignore_index if ignore_index is not None else torch.ones_like(t, dtype=torch.bool)
    return _np(p[keep]), _np(t[keep])


def _present(cm):
    tp = np.diag(cm)
    return (cm.sum(0) + cm.sum(1) - tp) > 0


def _ref_multiclass(kind, average, p, t, ignore_index=None):
    pp, tt = _mc_labels(p, t, ignore_index)
    labels = list(range(C))
    cm = skm.confusion_matrix(tt, pp, labels=labels)
    present = _present(cm)
    if ignore_index is not None and 0 <= ignore_index < C:
        present[ignore_index] = False if kind == "jaccard" else present[ignore_index]

    def per_class(vals, support):
        vals = np.asarray(vals, dtype=float)
        if average == "micro":
            raise AssertionError
        if average in (None, "none"):
            return vals
        if average == "weighted":
            w = support.astype(float)
            return (vals * w).sum() / w.sum() if w.sum() else 0.0
        return vals[present].mean() if present.any() else 0.0

    support = cm.sum(1)
    if kind in ("accuracy", "recall", "hamming"):
        if average == "micro":
            v = skm.accuracy_score(tt, pp) if kind != "recall" else skm.recall_score(tt, pp, average="micro", labels=labels, zero_division=0)
            return 1 - v if kind == "hamming" else v
        r = skm.recall_score(tt, pp, average=None, labels=labels, zero_division=0)
        r = 1 - r if kind == "hamming" else r
        return per_class(r, support)
    if kind in ("precision", "f1"):
        fn = skm.precision_score if kind == "precision" else skm.f1_score
        if average == "micro":
            return fn(tt, pp, average="micro", labels=labels, zero_division=0)
        return per_class(fn(tt, pp, average=None, labels=labels, zero_division=0), support)
    if kind == "specificity":
        tp = np.diag(cm)
        fp = cm.sum(0) - tp
        fn_ = cm.sum(1) - tp
        tn = cm.sum() - tp - fp - fn_
        if average == "micro":
            return tn.sum() / (tn.sum() + fp.sum())
        spec = np.where(tn + fp > 0, tn / np.maximum(tn + fp, 1), 0.0)
        return per_class(spec, support)
    if kind == "jaccard":
        if average == "micro":
            tp = np.diag(cm)
            un = cm.sum(0) + cm.sum(1) - tp
            if ignore_index is not None and 0 <= ignore_index < C:
                return tp.sum() / (un.sum() - un[ignore_index])
            return tp.sum() / un.sum()
        j = skm.jaccard_score(tt, pp, average=None, labels=labels, zero_division=0)
        return per_class(j, support)
    if kind == "confmat":
        return cm
    if kind == "kappa":
        return skm.cohen_kappa_score(tt, pp)
    if kind == "mcc":
        return skm.matthews_corrcoef(tt, pp)
    raise ValueError(kind)


def _ml_binarize(p):
    if p.is_floating_point():
        if not ((p >= 0) & (p <= 1)).all():
            p = p.sigmoid()
        p = (p > 0.5).long()
    return p


def _ref_multilabel(kind, average, p, t):
    pp = _np(_ml_binarize(p).reshape(-1, L))
    tt = _np(t.reshape(-1, L))
    if kind == "accuracy":
        if average == "micro":
            return (pp == tt).mean()
        per = (pp == tt).mean(0)
        if average == "weighted":
            w = tt.sum(0)
            return (per * w).sum() / w.sum()
        return per if average in (None, "none") else per.mean()
    fn = {"precision": skm.precision_score, "recall": skm.recall_score, "f1": skm.f1_score}[kind]
    return fn(tt, pp, average=None if average == "none" else average, zero_division=0)


# ------------------------------------------------------------------------------------------------------- tests
BIN_FUN = {
    "accuracy": (tm.BinaryAccuracy, F.binary_accuracy, {}),
    "precision": (tm.BinaryPrecision, F.binary_precision, {}),
    "recall": (tm.BinaryRecall, F.binary_recall, {}),
    "f1": (tm.BinaryF1Score, F.binary_f1_score, {}),
    "fbeta2": (tm.BinaryFBetaScore, partial(F.binary_fbeta_score, beta=2.0), {"beta": 2.0}),
    "hamming": (tm.BinaryHammingDistance, F.binary_hamming_distance, {}),
    "specificity": (tm.BinarySpecificity, F.binary_specificity, {}),
    "confmat": (tm.BinaryConfusionMatrix, F.binary_confusion_matrix, {}),
    "kappa": (tm.BinaryCohenKappa, F.binary_cohen_kappa, {}),
    "jaccard": (tm.BinaryJaccardIndex, F.binary_jaccard_index, {}),
    "mcc": (tm.BinaryMatthewsCorrCoef, F.binary_matthews_corrcoef, {}),
}


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit", "label"])
@pytest.mark.parametrize("name", list(BIN_FUN))
@pytest.mark.parametrize("ignore_index", [None, -1])
def test_binary(device, kind, name, ignore_index):
    p, t = _binary_inputs(kind)
    if ignore_index is not None:
        t[:, ::5] = ignore_index
    cls, fn, extra = BIN_FUN[name]
    ref = partial(_ref_binary, name, ignore_index=ignore_index)
    args = dict(extra, ignore_index=ignore_index)
    run_class_test(p, t, cls, ref, metric_args=args, device=device, atol=1e-5)
    run_functional_test(p, t, partial(fn, ignore_index=ignore_index), ref, device=device, atol=1e-5)


MC_FUN = {
    "accuracy": (tm.MulticlassAccuracy, F.multiclass_accuracy),
    "precision": (tm.MulticlassPrecision, F.multiclass_precision),
    "recall": (tm.MulticlassRecall, F.multiclass_recall),
    "f1": (tm.MulticlassF1Score, F.multiclass_f1_score),
    "hamming": (tm.MulticlassHammingDistance, F.multiclass_hamming_distance),
    "specificity": (tm.MulticlassSpecificity, F.multiclass_specificity),
    "jaccard": (tm.MulticlassJaccardIndex, F.multiclass_jaccard_index),
}


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["logit", "label"])
@pytest.mark.parametrize("name", list(MC_FUN))
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", "none"])
@pytest.mark.parametrize("ignore_index", [None, 0, -1])
def test_multiclass(device, kind, name, average, ignore_index):
    p, t = _multiclass_inputs(kind)
    if ignore_index is not None:
        t[:, ::5] = ignore_index
    cls, fn = MC_FUN[name]
    ref = partial(_ref_multiclass, name, average, ignore_index=ignore_index)
    args = {"num_classes": C, "average": average, "ignore_index": ignore_index}
    run_class_test(p, t, cls, ref, metric_args=args, device=device, atol=1e-5)
    run_functional_test(p, t, partial(fn, **args), ref, device=device, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name,cls,fn", [
    ("confmat", tm.MulticlassConfusionMatrix, F.multiclass_confusion_matrix),
    ("kappa", tm.MulticlassCohenKappa, F.multiclass_cohen_kappa),
    ("mcc", tm.MulticlassMatthewsCorrCoef, F.multiclass_matthews_corrcoef),
])
@pytest.mark.parametrize("ignore_index", [None, 1, -1])
def test_multiclass_confmat_family(device, name, cls, fn, ignore_index):
    p, t = _multiclass_inputs("logit")
    if ignore_index is not None:
        t[:, ::5] = ignore_index
    ref = partial(_ref_multiclass, name, None, ignore_index=ignore_index)
    args = {"num_classes": C, "ignore_index": ignore_index}
    run_class_test(p, t, cls, ref, metric_args=args, device=device, atol=1e-5)
    run_functional_test(p, t, partial(fn, **args), ref, device=device, atol=1e-5)


ML_FUN = {
    "accuracy": (tm.MultilabelAccuracy, F.multilabel_accuracy),
    "precision": (tm.MultilabelPrecision, F.multilabel_precision),
    "recall": (tm.MultilabelRecall, F.multilabel_recall),
    "f1": (tm.MultilabelF1Score, F.multilabel_f1_score),
}


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("kind", ["prob", "logit", "label"])
@pytest.mark.parametrize("name", list(ML_FUN))
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", "none"])
def test_multilabel(device, kind, name, average):
    p, t = _multilabel_inputs(kind)
    cls, fn = ML_FUN[name]
    ref = partial(_ref_multilabel, name, average)
    args = {"num_labels": L, "average": average}
    run_class_test(p, t, cls, ref, metric_args=args, device=device, atol=1e-5)
    run_functional_test(p, t, partial(fn, **args), ref, device=device, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_multilabel_confusion_matrix(device):
    p, t = _multilabel_inputs("prob")

    def ref(p, t):
        return skm.multilabel_confusion_matrix(_np(t.reshape(-1, L)), _np(_ml_binarize(p).reshape(-1, L)))

    run_class_test(p, t, tm.MultilabelConfusionMatrix, ref, metric_args={"num_labels": L}, device=device)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("top_k", [2, 3])
def test_multiclass_topk_accuracy(device, top_k):
    p, t = _multiclass_inputs("logit")

    def ref(p, t):
        return skm.top_k_accuracy_score(_np(t.flatten()), _np(p.reshape(-1, C)), k=top_k, labels=list(range(C)))

    run_class_test(p, t, tm.MulticlassAccuracy, ref, metric_args={"num_classes": C, "top_k": top_k, "average": "micro"},
                   device=device, atol=1e-5)


@pytest.mark.parametrize("device", DEVICES)
def test_samplewise_multidim(device):
    p = torch.randn(NB, BS, C, 6)
    t = torch.randint(0, C, (NB, BS, 6))

    def ref(p, t):
        labs = p.argmax(1)
        return torch.tensor([(labs[i] == t[i]).float().mean().item() for i in range(p.shape[0])])

    run_class_test(p, t, tm.MulticlassAccuracy,
                   ref, metric_args={"num_classes": C, "average": "micro", "multidim_average": "samplewise"},
                   device=device)


def test_task_wrappers():
    assert isinstance(tm.Accuracy(task="binary"), tm.BinaryAccuracy)
    assert isinstance(tm.Accuracy(task="multiclass", num_classes=3), tm.MulticlassAccuracy)
    assert isinstance(tm.F1Score(task="multilabel", num_labels=3), tm.MultilabelF1Score)
    assert isinstance(tm.ConfusionMatrix(task="multiclass", num_classes=3), tm.MulticlassConfusionMatrix)
    with pytest.raises(ValueError, match="Invalid Classification"):
        tm.Accuracy(task="nope")
    p, t = torch.randn(20, 3), torch.randint(0, 3, (20,))
    assert_close(F.accuracy(p, t, task="multiclass", num_classes=3), F.multiclass_accuracy(p, t, 3, average="micro"))


def test_validation_errors_cpu():
    m = tm.MulticlassAccuracy(num_classes=3)
    with pytest.raises(RuntimeError, match="unique values"):
        m.update(torch.randn(10, 3), torch.tensor([0, 1, 2, 5, 0, 1, 2, 0, 1, 2]))
    with pytest.raises(ValueError):
        tm.MulticlassAccuracy(num_classes=1)
    with pytest.raises(RuntimeError):
        F.binary_accuracy(torch.rand(10), torch.randint(2, 5, (10,)))


@pytest.mark.gpu
def test_validation_errors_deferred_gpu():
    m = tm.MulticlassAccuracy(num_classes=3).cuda()
    m.update(torch.randn(10, 3, device="cuda"), torch.tensor([0, 1, 2, 5, 0, 1, 2, 0, 1, 2], device="cuda"))
    with pytest.raises(RuntimeError, match="unique values"):
        m.compute()


@pytest.mark.ddp
@pytest.mark.parametrize("name", ["accuracy", "f1"])
def test_multiclass_ddp(name):
    p, t = _multiclass_inputs("logit")
    cls, _ = MC_FUN[name]
    run_ddp_class_test(p, t, cls, partial(_ref_multiclass, name, "macro"), metric_args={"num_classes": C})


@pytest.mark.ddp
def test_confmat_ddp():
    p, t = _multiclass_inputs("logit")
    run_ddp_class_test(p, t, tm.MulticlassConfusionMatrix, partial(_ref_multiclass, "confmat", None),
                       metric_args={"num_classes": C})
