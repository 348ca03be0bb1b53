"""Pearson / concordance per-rank merge as one kernel (``ops.corr_merge``, csrc/regression/regression_compute.hip)
against the reference's loop over ranks (S/regression/pearson.py:28-71, its formula written out here) and against the
statistics of the concatenated data."""
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional.regression.correlation import _final_aggregation


def _ref_loop(means_x, means_y, vars_x, vars_y, corrs_xy, nbs):
    mx1, my1, vx1, vy1, cxy1, n1 = (t[0].clone() for t in (means_x, means_y, vars_x, vars_y, corrs_xy, nbs))
    for i in range(1, len(means_x)):
        mx2, my2, vx2, vy2, cxy2, n2 = (t[i].clone() for t in (means_x, means_y, vars_x, vars_y, corrs_xy, nbs))
        nb = n1 + n2
        mean_x = (n1 * mx1 + n2 * mx2) / nb
        mean_y = (n1 * my1 + n2 * my2) / nb
        ex1 = (n1 + 1) * mean_x - n1 * mx1
        vx1 += (ex1 - mx1) * (ex1 - mean_x) - (ex1 - mean_x) ** 2
        ex2 = (n2 + 1) * mean_x - n2 * mx2
        vx2 += (ex2 - mx2) * (ex2 - mean_x) - (ex2 - mean_x) ** 2
        var_x = vx1 + vx2
        ey1 = (n1 + 1) * mean_y - n1 * my1
        vy1 += (ey1 - my1) * (ey1 - mean_y) - (ey1 - mean_y) ** 2
        ey2 = (n2 + 1) * mean_y - n2 * my2
        vy2 += (ey2 - my2) * (ey2 - mean_y) - (ey2 - mean_y) ** 2
        var_y = vy1 + vy2
        cxy1 += (ex1 - mx1) * (ey1 - mean_y) - (ex1 - mean_x) * (ey1 - mean_y)
        cxy2 += (ex2 - mx2) * (ey2 - mean_y) - (ex2 - mean_x) * (ey2 - mean_y)
        corr_xy = cxy1 + cxy2
        mx1, my1, vx1, vy1, cxy1, n1 = mean_x, mean_y, var_x, var_y, corr_xy, nb
    return mx1, my1, vx1, vy1, cxy1, n1


def _rank_states(w, k, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    parts = []
    for r in range(w):
        n = 5 + 7 * r
        x = torch.randn(n, k, generator=g, dtype=torch.float64) * (r + 1) + r
        y = 0.5 * x + torch.randn(n, k, generator=g, dtype=torch.float64)
        mx, my = x.mean(0), y.mean(0)
        parts.append((x, y, [mx, my, ((x - mx) ** 2).sum(0), ((y - my) ** 2).sum(0), ((x - mx) * (y - my)).sum(0),
                             torch.full((k,), float(n), dtype=torch.float64)]))
    stacked = [torch.stack([p[2][i] for p in parts]).to(dtype) for i in range(6)]
    x = torch.cat([p[0] for p in parts])
    y = torch.cat([p[1] for p in parts])
    return stacked, x, y


@pytest.mark.parametrize("w", [1, 2, 3, 8])
@pytest.mark.parametrize("k", [1, 5])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_corr_merge_matches_reference_loop(w, k, dtype, device):
    stacked, x, y = _rank_states(w, k, dtype)
    ref = _ref_loop(*[s.double() for s in stacked])
    out = _final_aggregation(*[s.to(device) for s in stacked])
    tol = dict(rtol=1e-5, atol=1e-4) if dtype == torch.float32 else dict(rtol=1e-10, atol=1e-9)
    for a, b in zip(out, ref):
        assert a.dtype == dtype and a.device.type == device
        torch.testing.assert_close(a.cpu().double(), b, **tol)
    # and the statistics of the concatenated data
    mx, my = x.mean(0), y.mean(0)
    torch.testing.assert_close(out[2].cpu().double(), ((x - mx) ** 2).sum(0), **tol)
    torch.testing.assert_close(out[4].cpu().double(), ((x - mx) * (y - my)).sum(0), **tol)


def test_corr_merge_single_launch_shape():
    stacked, _, _ = _rank_states(4, 3, torch.float32)
    merged = ops.corr_merge(torch.stack(stacked))
    assert merged.shape == (6, 3)
    scalar = _final_aggregation(*[s[:, 0] for s in stacked])
    assert all(t.shape == () for t in scalar)
