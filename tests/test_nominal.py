"""Nominal association metrics vs scipy / numpy oracles (reference ``tests/unittests/nominal``; dython and
statsmodels are not installed, so bias-corrected variants, Theil's U and Fleiss' kappa use plain numpy oracles of the
textbook formulas)."""
import itertools

import numpy as np
import pytest
import torch
from scipy.stats import chi2_contingency
from scipy.stats.contingency import association

from torchmetrics_amd import functional as F
from torchmetrics_amd.nominal import CramersV, FleissKappa, PearsonsContingencyCoefficient, TheilsU, TschuprowsT

_g = torch.Generator().manual_seed(3)
NB, BS, K = 3, 100, 4
PREDS = torch.randint(0, K, (NB, BS), generator=_g)
TARGET = torch.randint(0, K, (NB, BS), generator=_g)
MATRIX = torch.randint(0, 4, (200, 5), generator=_g)


def _table(p, t):
    p, t = np.asarray(p), np.asarray(t)
    cm = np.zeros((int(max(p.max(), t.max())) + 1,) * 2)
    np.add.at(cm, (t, p), 1)
    cm = cm[cm.sum(1) > 0]
    return cm[:, cm.sum(0) > 0]


def _np_assoc(p, t, kind, bias):
    cm = _table(p, t)
    n = cm.sum()
    chi2 = chi2_contingency(cm, correction=bias)[0] if min(cm.shape) > 1 else 0.0
    phi2 = chi2 / n
    r, c = cm.shape
    if kind == "pearson":
        return np.sqrt(phi2 / (1 + phi2))
    if bias:
        phi2 = max(0.0, phi2 - (r - 1) * (c - 1) / (n - 1))
        r, c = r - (r - 1) ** 2 / (n - 1), c - (c - 1) ** 2 / (n - 1)
    if kind == "cramer":
        return min(1.0, np.sqrt(phi2 / min(r - 1, c - 1)))
    return min(1.0, np.sqrt(phi2 / np.sqrt((r - 1) * (c - 1))))


def _np_theils_u(p, t):
    cm = _table(p, t)
    n = cm.sum()
    pxy = cm / n
    py = cm.sum(1, keepdims=True) / n
    with np.errstate(divide="ignore", invalid="ignore"):
        sxy = np.nansum(pxy * np.log(py / pxy))
    px = cm.sum(0) / n
    sx = -np.sum(px * np.log(px))
    return 0.0 if sx == 0 else (sx - sxy) / sx


def _np_fleiss(counts):
    counts = np.asarray(counts, dtype=np.float64)
    n = counts.sum(1).max()
    p_i = counts.sum(0) / (counts.shape[0] * n)
    p_j = ((counts**2).sum(1) - n) / (n * (n - 1))
    pe = (p_i**2).sum()
    return (p_j.mean() - pe) / (1 - pe + 1e-5)


def test_scipy_association_unbiased():
    for i in range(NB):
        cm = _table(PREDS[i], TARGET[i]).astype(np.int64)
        for kind, fn in (("cramer", F.cramers_v), ("tschuprow", F.tschuprows_t)):
            got = fn(PREDS[i], TARGET[i], bias_correction=False).item()
            assert np.isclose(got, association(cm, method=kind, correction=False), atol=1e-6)
        got = F.pearsons_contingency_coefficient(PREDS[i], TARGET[i]).item()
        assert np.isclose(got, association(cm, method="pearson", correction=False), atol=1e-6)


@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize(
    ("cls", "fn", "kind"),
    [(CramersV, F.cramers_v, "cramer"), (TschuprowsT, F.tschuprows_t, "tschuprow"),
     (PearsonsContingencyCoefficient, F.pearsons_contingency_coefficient, "pearson")],
)
def test_chi2_family(cls, fn, kind, bias):
    kw = {} if kind == "pearson" else {"bias_correction": bias}
    for i in range(NB):
        assert np.isclose(fn(PREDS[i], TARGET[i], **kw).item(), _np_assoc(PREDS[i], TARGET[i], kind, bias), atol=1e-6)
    m = cls(num_classes=K, **kw)
    for i in range(NB):
        m.update(PREDS[i], TARGET[i])
    assert np.isclose(m.compute().item(), _np_assoc(PREDS.flatten(), TARGET.flatten(), kind, bias), atol=1e-6)


def test_yates_2x2():
    p = torch.tensor([0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 1])
    t = torch.tensor([0, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1])
    for bias in (True, False):
        assert np.isclose(F.cramers_v(p, t, bias_correction=bias).item(), _np_assoc(p, t, "cramer", bias), atol=1e-6)


def test_theils_u():
    for i in range(NB):
        assert np.isclose(F.theils_u(PREDS[i], TARGET[i]).item(), _np_theils_u(PREDS[i], TARGET[i]), atol=1e-6)
    m = TheilsU(num_classes=K)
    for i in range(NB):
        m.update(PREDS[i], TARGET[i])
    assert np.isclose(m.compute().item(), _np_theils_u(PREDS.flatten(), TARGET.flatten()), atol=1e-6)


@pytest.mark.parametrize(
    ("fn", "oracle", "sym"),
    [
        (F.cramers_v_matrix, lambda x, y: _np_assoc(x, y, "cramer", True), True),
        (F.tschuprows_t_matrix, lambda x, y: _np_assoc(x, y, "tschuprow", True), True),
        (F.pearsons_contingency_coefficient_matrix, lambda x, y: _np_assoc(x, y, "pearson", False), True),
        (F.theils_u_matrix, _np_theils_u, False),
    ],
)
def test_matrix_variants(fn, oracle, sym):
    out = fn(MATRIX)
    v = MATRIX.shape[1]
    ref = np.ones((v, v))
    for i, j in itertools.combinations(range(v), 2):
        ref[i, j] = oracle(MATRIX[:, i], MATRIX[:, j])
        ref[j, i] = ref[i, j] if sym else oracle(MATRIX[:, j], MATRIX[:, i])
    assert np.allclose(out.numpy(), ref, atol=1e-6)


def test_nan_strategies():
    p = torch.tensor([0.0, 1, 2, float("nan"), 1, 0, 2, 2, 1, 0])
    t = torch.tensor([0.0, 1, 1, 2, float("nan"), 0, 2, 1, 1, 2])
    keep = ~(p.isnan() | t.isnan())
    got = F.cramers_v(p, t, nan_strategy="drop").item()
    assert np.isclose(got, _np_assoc(p[keep].long(), t[keep].long(), "cramer", True), atol=1e-6, equal_nan=True)
    got = F.tschuprows_t(p, t, bias_correction=False, nan_strategy="replace", nan_replace_value=0.0).item()
    assert np.isclose(got, _np_assoc(p.nan_to_num(0).long(), t.nan_to_num(0).long(), "tschuprow", False), atol=1e-6)
    m = torch.stack([p, t, torch.tensor([0.0, 1, 1, 0, 1, 0, 0, 1, 1, 0])], 1)
    out = F.cramers_v_matrix(m, nan_strategy="drop")
    assert np.isclose(out[0, 1].item(), F.cramers_v(p, t, nan_strategy="drop").item(), atol=1e-6, equal_nan=True)
    with pytest.raises(ValueError, match="nan_strategy"):
        F.cramers_v(p, t, nan_strategy="foo")


def test_fleiss_kappa():
    counts = torch.randint(0, 4, (20, 5), generator=_g)
    counts[:, -1] = 10 - counts[:, :-1].sum(1).clamp(max=10)
    counts[:, -1] = counts[:, -1].clamp(min=0)
    assert np.isclose(F.fleiss_kappa(counts).item(), _np_fleiss(counts), atol=1e-6)
    probs = torch.randn(20, 3, 7, generator=_g)
    oh = torch.nn.functional.one_hot(probs.argmax(1), 3).sum(1)
    assert np.isclose(F.fleiss_kappa(probs, mode="probs").item(), _np_fleiss(oh), atol=1e-6)
    m = FleissKappa(mode="probs")
    m.update(probs[:10])
    m.update(probs[10:])
    assert np.isclose(m.compute().item(), _np_fleiss(oh), atol=1e-6)


@pytest.mark.gpu
def test_nominal_gpu():
    for cls, kind in ((CramersV, "cramer"), (TschuprowsT, "tschuprow"), (PearsonsContingencyCoefficient, "pearson")):
        kw = {} if kind == "pearson" else {"bias_correction": True}
        m = cls(num_classes=K, **kw).cuda()
        for i in range(NB):
            m.update(PREDS[i].cuda(), TARGET[i].cuda())
        bias = kind != "pearson"
        assert np.isclose(m.compute().item(), _np_assoc(PREDS.flatten(), TARGET.flatten(), kind, bias), atol=1e-6)
    out = F.theils_u_matrix(MATRIX.cuda()).cpu()
    assert np.isclose(out[0, 1].item(), _np_theils_u(MATRIX[:, 0], MATRIX[:, 1]), atol=1e-6)
    m = CramersV(num_classes=2).cuda()
    m.update(torch.tensor([0, 5], device="cuda"), torch.tensor([0, 1], device="cuda"))
    with pytest.raises((ValueError, RuntimeError)):
        m.compute()
