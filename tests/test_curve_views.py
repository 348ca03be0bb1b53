"""Unbinned multiclass / multilabel ROC and PR curves: every class's tensors are views of one epilogue buffer
(``functional/classification/_sorted.py`` ``roc_curves`` / ``pr_curves``) and equal the per-class chain of the
reference (``F/classification/roc.py:107-112``, ``F/classification/precision_recall_curve.py:356-371``), degenerate
classes (no positives) included, warnings and dtypes too."""
import warnings

import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification.precision_recall_curve import (
    _clf_curves,
    _clf_pr_curves,
    _pr_from_clf,
)
from torchmetrics_amd.functional.classification.roc import _clf_roc_curves, _roc_from_clf

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _per_class(p, t, tmode):
    fl, tl, hl, host = _clf_curves(p, t, tmode)
    roc = [_roc_from_clf(f, tp, th, h[1], h[0]) for f, tp, th, h in zip(fl, tl, hl, host)]
    pr = [_pr_from_clf(f, tp, th) for f, tp, th in zip(fl, tl, hl)]
    return roc, pr


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tmode", ["ovr", "elem"])
def test_curve_views_match_per_class_chain(device, dtype, tmode):
    g = torch.Generator().manual_seed(3)
    m, c = 400, 6
    p = torch.rand(m, c, generator=g)
    p[::3] = p[::3].round(decimals=1)  # ties
    p = p.to(dtype).to(device)
    if tmode == "ovr":
        t, mode = torch.randint(0, c - 1, (m,), generator=g).to(device), ops.CLF_T_OVR  # class c-1: no positives
    else:
        t, mode = torch.randint(0, 2, (m, c), generator=g), ops.CLF_T_ELEM
        t[:, 2] = 0
        t = t.to(device)
    with warnings.catch_warnings(record=True) as w_old:
        warnings.simplefilter("always")
        roc_old, pr_old = _per_class(p, t, mode)
    with warnings.catch_warnings(record=True) as w_new:
        warnings.simplefilter("always")
        roc_new = _clf_roc_curves(p, t, mode)
        pr_new = _clf_pr_curves(p, t, mode)
    assert [str(x.message) for x in w_old] == [str(x.message) for x in w_new]
    for i in range(c):
        for k in range(3):
            a, b = roc_old[i][k], roc_new[k][i]
            assert a.dtype == b.dtype and torch.equal(a, b), (i, k)
            a, b = pr_old[i][k], pr_new[k][i]
            assert a.dtype == b.dtype and torch.equal(a.nan_to_num(-7.0), b.nan_to_num(-7.0)), (i, k)
    # the curves of non-degenerate classes share one storage per output
    base = roc_new[2][0].untyped_storage().data_ptr()
    assert all(x.untyped_storage().data_ptr() == base for x in roc_new[2])
    base = pr_new[0][0].untyped_storage().data_ptr()
    assert all(x.untyped_storage().data_ptr() == base for x in pr_new[0])
