"""GPU reductions pinned to external oracles instead of this package's own CPU formulation: the fused confusion-matrix
reductions (Jaccard / Cohen kappa / MCC, ``csrc/classification/confmat_reduce.hip``) against sklearn, the binned
calibration error against a numpy transcription of the reference's binning formula (``F/classification/
calibration_error.py:60-108``; sklearn has no ECE), and the fused regression computes (R2 / explained variance /
Pearson / Spearman-free paths, ``csrc/regression/regression_compute.hip``) against sklearn and scipy."""
import numpy as np
import pytest
import torch
from scipy.stats import pearsonr
from sklearn.metrics import cohen_kappa_score, explained_variance_score, jaccard_score, matthews_corrcoef, r2_score

import torchmetrics_amd as tm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _labels(n, c, seed, missing=None):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, c, (n,), generator=g)
    p = torch.where(torch.rand(n, generator=g) < 0.6, t, torch.randint(0, c, (n,), generator=g))
    if missing is not None:
        p[p == missing] = (missing + 1) % c
        t[t == missing] = (missing + 1) % c
    return p, t


@pytest.mark.parametrize("c,missing", [(2, None), (5, None), (10, 7), (101, 3)])
def test_confmat_reductions_vs_sklearn(c, missing):
    p, t = _labels(200_000, c, c, missing)
    pn, tn = p.numpy(), t.numpy()
    labels = list(range(c))
    for avg in ("micro", "macro", "weighted"):
        m = tm.classification.MulticlassJaccardIndex(c, average=avg).to(DEV)
        m.update(p.to(DEV), t.to(DEV))
        # the reference's macro mean skips classes absent from both preds and target (F/classification/jaccard.py
        # `_jaccard_index_reduce`: zero weight): sklearn over the present labels
        lab = np.union1d(pn, tn).tolist() if avg == "macro" else labels
        ref = jaccard_score(tn, pn, labels=lab, average=avg, zero_division=0)
        np.testing.assert_allclose(float(m.compute()), ref, rtol=1e-5, atol=1e-6)
    for w in (None, "linear", "quadratic"):
        m = tm.classification.MulticlassCohenKappa(c, weights=w).to(DEV)
        m.update(p.to(DEV), t.to(DEV))
        # labels=all classes: weights by class index over the full C x C table, as the reference's confusion matrix
        np.testing.assert_allclose(float(m.compute()), cohen_kappa_score(tn, pn, labels=labels, weights=w),
                                   rtol=1e-5, atol=1e-6)
    m = tm.classification.MulticlassMatthewsCorrCoef(c).to(DEV)
    m.update(p.to(DEV), t.to(DEV))
    np.testing.assert_allclose(float(m.compute()), matthews_corrcoef(tn, pn), rtol=1e-5, atol=1e-6)


def _ece_numpy(conf, acc, n_bins, norm):
    """The reference's binning (``_binning_bucketize``: bucketize(right=True) - 1 over linspace(0, 1, n_bins + 1),
    the top boundary in the last bin) and l1 / l2 / max norms, in float64 numpy."""
    bounds = np.linspace(0, 1, n_bins + 1)
    idx = np.clip(np.searchsorted(bounds, conf, side="right") - 1, 0, n_bins - 1)
    cnt = np.bincount(idx, minlength=n_bins).astype(np.float64)
    s_conf = np.bincount(idx, weights=conf, minlength=n_bins)
    s_acc = np.bincount(idx, weights=acc, minlength=n_bins)
    nz = cnt > 0
    gap = np.zeros(n_bins)
    gap[nz] = np.abs(s_acc[nz] / cnt[nz] - s_conf[nz] / cnt[nz])
    prop = cnt / cnt.sum()
    if norm == "l1":
        return float((gap * prop).sum())
    if norm == "max":
        return float(gap.max())
    return float(np.sqrt((gap**2 * prop).sum()))


@pytest.mark.parametrize("n_bins", [5, 15, 100])
@pytest.mark.parametrize("norm", ["l1", "l2", "max"])
def test_calibration_error_vs_numpy_formula(n_bins, norm):
    g = torch.Generator().manual_seed(n_bins)
    logits = torch.randn(100_000, 6, generator=g) * 2
    t = torch.randint(0, 6, (100_000,), generator=g)
    m = tm.classification.MulticlassCalibrationError(6, n_bins=n_bins, norm=norm).to(DEV)
    for lo in range(0, 100_000, 25_000):
        m.update(logits[lo:lo + 25_000].to(DEV), t[lo:lo + 25_000].to(DEV))
    prob = torch.softmax(logits.double(), -1)
    conf, pred = prob.max(-1)
    ref = _ece_numpy(conf.numpy(), (pred == t).double().numpy(), n_bins, norm)
    np.testing.assert_allclose(float(m.compute()), ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("k", [1, 3])
def test_regression_computes_vs_sklearn_scipy(k):
    g = torch.Generator().manual_seed(k)
    x = torch.randn(300_000, k, generator=g) * 3 + 1
    y = 0.7 * x + torch.randn(300_000, k, generator=g)
    if k == 1:
        x, y = x[:, 0], y[:, 0]
    ms = {"r2": tm.regression.R2Score(num_outputs=k), "ev": tm.regression.ExplainedVariance(multioutput="raw_values"),
          "pearson": tm.regression.PearsonCorrCoef(num_outputs=k)}
    ms = {n: m.to(DEV) for n, m in ms.items()}
    for lo in range(0, 300_000, 60_000):
        for m in ms.values():
            m.update(x[lo:lo + 60_000].to(DEV), y[lo:lo + 60_000].to(DEV))
    xn, yn = x.double().numpy(), y.double().numpy()
    np.testing.assert_allclose(float(ms["r2"].compute()), r2_score(yn, xn), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ms["ev"].compute().cpu().double().numpy().reshape(-1),
                               np.atleast_1d(explained_variance_score(yn, xn, multioutput="raw_values")),
                               rtol=1e-5, atol=1e-6)
    pr = ms["pearson"].compute().cpu().double().numpy().reshape(-1)
    ref = [pearsonr(xn, yn)[0]] if k == 1 else [pearsonr(xn[:, j], yn[:, j])[0] for j in range(k)]
    np.testing.assert_allclose(pr, ref, rtol=1e-5, atol=1e-6)
