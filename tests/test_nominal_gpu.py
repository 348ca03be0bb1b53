"""Nominal association metrics on the per-table statistics kernel (``csrc/nominal/table_stats.hip``) vs the CPU
formulation and scipy (``scipy.stats.contingency.association``, ``chi2_contingency``)."""
import numpy as np
import pytest
import torch
from scipy.stats import chi2_contingency
from scipy.stats.contingency import association

from torchmetrics_amd import ops
from torchmetrics_amd.functional import nominal as N

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _data(n, k, seed, empty=()):
    g = torch.Generator().manual_seed(seed)
    p = torch.randint(0, k, (n,), generator=g)
    t = (p + torch.randint(0, 3, (n,), generator=g)) % k
    for e in empty:  # categories that never occur (masked rows / columns)
        p[p == e] = (e + 1) % k
        t[t == e] = (e + 2) % k
    return p, t


@pytest.mark.parametrize("k,n,empty", [(2, 500, ()), (5, 10000, (3,)), (37, 200000, (0, 11)), (300, 1_000_000, ())])
def test_table_stats_kernel_vs_torch(k, n, empty):
    p, t = _data(n, k, k, empty)
    cm = torch.zeros(k, k, dtype=torch.long)
    cm.index_put_((t, p), torch.ones(n, dtype=torch.long), accumulate=True)
    got = ops.nominal_table_stats(cm[None].to(DEV)).cpu()[0]
    ref = N._TableStats._torch_stats(cm[None].double())[0]
    torch.testing.assert_close(got, ref, rtol=1e-9, atol=1e-9)
    # scipy pins chi^2 (with / without the Yates correction) on the compacted table
    c = cm.numpy()
    c = c[c.sum(1) > 0][:, c.sum(0) > 0]
    st = N._TableStats(cm[None].to(DEV))
    for corr in (False, True):
        chi = chi2_contingency(c, correction=corr)[0] if min(c.shape) > 1 else 0.0
        np.testing.assert_allclose(float(st.chi_squared(corr)[0]), chi, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("k", [2, 6, 40])
def test_functionals_gpu_vs_cpu_and_scipy(k):
    p, t = _data(50000, k, 100 + k)
    for fn in (N.cramers_v, N.tschuprows_t, N.pearsons_contingency_coefficient, N.theils_u):
        kw = {} if fn in (N.pearsons_contingency_coefficient, N.theils_u) else {"bias_correction": False}
        got = fn(p.to(DEV), t.to(DEV), **kw).cpu()
        ref = fn(p, t, **kw)
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    cm = torch.zeros(k, k, dtype=torch.long)
    cm.index_put_((t, p), torch.ones(len(p), dtype=torch.long), accumulate=True)
    c = cm.numpy()
    for fn, method in ((N.cramers_v, "cramer"), (N.tschuprows_t, "tschuprow"), (N.pearsons_contingency_coefficient,
                                                                            "pearson")):
        kw = {} if method == "pearson" else {"bias_correction": False}
        np.testing.assert_allclose(float(fn(p.to(DEV), t.to(DEV), **kw)), association(c, method=method,
                                   correction=False), rtol=1e-5)


def test_matrix_variants_gpu_vs_cpu():
    g = torch.Generator().manual_seed(5)
    m = torch.randint(0, 7, (20000, 6), generator=g)
    m[:, 3] = (m[:, 0] + torch.randint(0, 2, (20000,), generator=g)) % 7
    for fn in (N.cramers_v_matrix, N.tschuprows_t_matrix, N.pearsons_contingency_coefficient_matrix,
               N.theils_u_matrix):
        got = fn(m.to(DEV)).cpu()
        ref = fn(m)
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6, equal_nan=True)
