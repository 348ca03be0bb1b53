"""average="macro" ROC / precision-recall curves: one batched interpolation (``ops.interp_mean``,
``csrc/classification/curve_interp.hip``) against the reference's algorithm written out as a per-class loop
(F/classification/roc.py:189-200, precision_recall_curve.py:566-580, utilities/compute.py:134-157) -- bit-identical,
binned and unbinned, including per-class precision curves that are not monotone (the segment is the reference's COUNT
``sum(x >= xp) - 1``, not a search, so it differs from torch.searchsorted there)."""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops


def _ref_interp(x, xp, fp):
    den = xp[1:] - xp[:-1]
    den[den == 0.0] = 1
    m = (fp[1:] - fp[:-1]) / den
    b = fp[:-1] - (m * xp[:-1])
    idx = torch.sum(torch.ge(x[:, None], xp[None, :]), 1) - 1  # S/utilities/compute.py:154, verbatim formula
    idx = torch.clamp(idx, 0, len(m) - 1)
    return m[idx] * x + b[idx]


def _ref_macro(xs, ys, thr, descending):
    grid = torch.cat(list(xs)).sort().values
    acc = torch.zeros_like(grid)
    for x, y in zip(xs, ys):
        acc += _ref_interp(grid, x, y)
    return grid, acc / len(xs), torch.cat(list(thr)).sort(descending=descending).values


def _data(n=600, c=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, c, generator=g).softmax(-1), torch.randint(0, c, (n,), generator=g)


@pytest.mark.parametrize("thresholds", [None, 11, 100])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_macro_roc_matches_reference_algorithm(thresholds, device):
    p, t = _data()
    fpr, tpr, thr = tm.functional.multiclass_roc(p.to(device), t.to(device), 6, thresholds=thresholds)
    thr_l = [thr] * 6 if isinstance(thr, torch.Tensor) else thr
    ref = _ref_macro([f.cpu() for f in fpr], [q.cpu() for q in tpr], [h.cpu() for h in thr_l], True)
    out = tm.functional.multiclass_roc(p.to(device), t.to(device), 6, thresholds=thresholds, average="macro")
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("thresholds", [None, 11])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_macro_pr_matches_reference_algorithm(thresholds, device):
    p, t = _data(seed=1)
    prec, rec, thr = tm.functional.multiclass_precision_recall_curve(p.to(device), t.to(device), 6,
                                                                      thresholds=thresholds)
    thr_l = [thr] * 6 if isinstance(thr, torch.Tensor) else thr
    assert any(not bool((q[1:] >= q[:-1]).all()) for q in prec)  # non-monotone precision curves are exercised
    ref = _ref_macro([q.cpu() for q in prec], [r.cpu() for r in rec], [h.cpu() for h in thr_l], False)
    out = tm.functional.multiclass_precision_recall_curve(p.to(device), t.to(device), 6, thresholds=thresholds,
                                                          average="macro")
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_interp_mean_ragged(dtype, device):
    g = torch.Generator().manual_seed(3)
    xs = [torch.rand(n, generator=g, dtype=dtype) for n in (2, 7, 50, 3)]
    xs[1] = xs[1].sort().values
    ys = [torch.rand(x.numel(), generator=g, dtype=dtype) for x in xs]
    xs[2][10] = xs[2][11]  # a zero-width segment
    grid = torch.cat([torch.cat(xs), torch.tensor([-1.0, 2.0], dtype=dtype)]).sort().values
    off = torch.tensor([0, 2, 9, 59, 62])
    out = ops.interp_mean(grid.to(device), torch.cat(xs).to(device), torch.cat(ys).to(device), off.to(device))
    ref = torch.zeros_like(grid)
    for x, y in zip(xs, ys):
        ref += _ref_interp(grid, x, y)
    assert torch.equal(out.cpu(), ref / 4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_interp_count_segment_non_monotone(dtype, device):
    """xp = [0.5, 0.3, 0.8] at v = 0.4: the reference's count picks segment 0 (one xp <= v), a search would pick 1."""
    xp = torch.tensor([0.5, 0.3, 0.8], dtype=dtype)
    fp = torch.tensor([1.0, 2.0, 4.0], dtype=dtype)
    grid = torch.tensor([-1.0, 0.3, 0.4, 0.5, 0.6, 0.8, 2.0], dtype=dtype)
    ref = _ref_interp(grid, xp, fp)
    out = ops.interp_mean(grid.to(device), xp.to(device), fp.to(device), torch.tensor([0, 3]).to(device))
    assert torch.equal(out.cpu(), ref)
    assert torch.equal(tm.utilities.compute.interp(grid, xp, fp), ref)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_interp_nan_and_random_non_monotone(device):
    g = torch.Generator().manual_seed(7)
    xs = [torch.rand(n, generator=g, dtype=torch.float64) for n in (5, 40, 2, 17)]
    xs[1][3] = float("nan")
    ys = [torch.rand(x.numel(), generator=g, dtype=torch.float64) for x in xs]
    grid = torch.cat([torch.rand(200, generator=g, dtype=torch.float64), torch.tensor([float("nan"), float("inf")],
                                                                                     dtype=torch.float64)])
    ref = torch.zeros_like(grid)
    for x, y in zip(xs, ys):
        ref += _ref_interp(grid, x, y)
        assert torch.equal(tm.utilities.compute.interp(grid, x, y), _ref_interp(grid, x, y), ) or torch.allclose(
            tm.utilities.compute.interp(grid, x, y), _ref_interp(grid, x, y), equal_nan=True)
    off = torch.tensor([0, 5, 45, 47, 64])
    out = ops.interp_mean(grid.to(device), torch.cat(xs).to(device), torch.cat(ys).to(device), off.to(device))
    assert torch.allclose(out.cpu(), ref / 4, equal_nan=True, rtol=0, atol=0)
