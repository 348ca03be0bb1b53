"""Spearman average ranks and Kendall statistics kernels vs scipy (CPU contract + ROCm kernels)."""
import numpy as np
import pytest
import torch
from scipy import stats

import torchmetrics_amd.functional as F
from torchmetrics_amd import ops

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n,levels", [(500, 0), (3000, 11), (20000, 50)])
@pytest.mark.parametrize("variant", ["b", "c"])
def test_kendall_vs_scipy(device, n, levels, variant):
    g = torch.Generator().manual_seed(n + levels)
    x = torch.randn(n, generator=g, dtype=torch.float64)
    y = x + torch.randn(n, generator=g, dtype=torch.float64)
    if levels:
        x, y = (x * levels / 4).round(), (y * levels / 4).round()
    tau = F.kendall_rank_corrcoef(x.to(device), y.to(device), variant=variant)
    ref = stats.kendalltau(x.numpy(), y.numpy(), variant=variant).statistic
    np.testing.assert_allclose(float(tau), ref, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("device", DEVICES)
def test_kendall_stats_multi_column_ties(device):
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(4000, 3, generator=g) * 3).round()
    y = (torch.randn(4000, 3, generator=g) * 3).round()
    st = ops.kendall_stats(x.to(device), y.to(device)).cpu()
    for c in range(3):
        xs, ys = x[:, c].numpy(), y[:, c].numpy()
        _, cx = np.unique(xs, return_counts=True)
        _, cy = np.unique(ys, return_counts=True)
        _, cxy = np.unique(np.stack([xs, ys], 1), axis=0, return_counts=True)
        assert st[c, 1] == (cx * (cx - 1) / 2).sum() and st[c, 4] == (cy * (cy - 1) / 2).sum()
        assert st[c, 2] == (cx * (cx - 1) * (cx - 2)).sum() and st[c, 6] == (cy * (cy - 1) * (2 * cy + 5)).sum()
        assert st[c, 7] == (cxy * (cxy - 1) / 2).sum()
        assert st[c, 8] == len(cx) and st[c, 9] == len(cy)
        # discordant pairs: strict (x, y) disagreements
        sx, sy = np.sign(xs[:, None] - xs[None]), np.sign(ys[:, None] - ys[None])
        assert st[c, 0] == ((sx * sy) < 0).sum() // 2


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("shape", [(1000,), (5000, 3)])
def test_spearman_vs_scipy(device, shape):
    g = torch.Generator().manual_seed(4)
    x = (torch.randn(*shape, generator=g) * 5).round()
    y = x + torch.randn(*shape, generator=g) * 3
    r = F.spearman_corrcoef(x.to(device), y.to(device)).cpu()
    if len(shape) == 1:
        np.testing.assert_allclose(float(r), stats.spearmanr(x.numpy(), y.numpy()).statistic, rtol=1e-5)
    else:
        for c in range(shape[1]):
            np.testing.assert_allclose(float(r[c]), stats.spearmanr(x[:, c].numpy(), y[:, c].numpy()).statistic,
                                       rtol=1e-5)


@pytest.mark.gpu
def test_kendall_large_n_gpu():
    g = torch.Generator().manual_seed(5)
    n = 200_000
    x = torch.randn(n, generator=g, dtype=torch.float64)
    y = (x + torch.randn(n, generator=g, dtype=torch.float64)).round(decimals=1)
    tau = F.kendall_rank_corrcoef(x.cuda(), y.cuda())
    np.testing.assert_allclose(float(tau), stats.kendalltau(x.numpy(), y.numpy()).statistic, rtol=1e-9)
