"""Clustering / nominal kernels (``csrc/clustering/cluster.hip``) pinned to scikit-learn at N = 10^7 labels
(extrinsic scores) and 10^6 x 8 points (intrinsic scores)."""
import numpy as np
import pytest
import torch

from torchmetrics_amd import ops
from torchmetrics_amd.functional import clustering as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
sk = pytest.importorskip("sklearn.metrics")


def _labels(n, k, seed, offset=0, gap=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, k, (n,), generator=g) * gap + offset


@pytest.mark.parametrize("offset,gap", [(0, 1), (-7, 3), (1000, 1)])
def test_contingency_matches_sklearn(offset, gap):
    from sklearn.metrics.cluster import contingency_matrix

    t = _labels(200_000, 12, 1, offset, gap)
    p = _labels(200_000, 9, 2, -offset, 1)
    got = ops.contingency(p.to(DEV), t.to(DEV)).cpu().numpy()
    exp = contingency_matrix(t.numpy(), p.numpy())
    np.testing.assert_array_equal(got, exp)


def test_contingency_sparse_range_falls_back():
    t = torch.tensor([0, 10**12, 5, 5, 10**12], dtype=torch.int64)
    p = torch.tensor([1, 1, 2, 3, 3], dtype=torch.int64)
    from sklearn.metrics.cluster import contingency_matrix

    np.testing.assert_array_equal(ops.contingency(p.to(DEV), t.to(DEV)).cpu().numpy(),
                                  contingency_matrix(t.numpy(), p.numpy()))


def test_extrinsic_scores_at_1e7():
    n = 10_000_000
    t = _labels(n, 20, 3)
    # predictions correlated with the target: 70 % copied (relabelled), the rest random
    g = torch.Generator().manual_seed(4)
    p = torch.where(torch.rand(n, generator=g) < 0.7, (t * 7 + 3) % 25, torch.randint(0, 25, (n,), generator=g))
    td, pd = t.to(DEV), p.to(DEV)
    tn, pn = t.numpy(), p.numpy()
    cases = [
        (F.mutual_info_score, sk.mutual_info_score),
        (F.adjusted_rand_score, sk.adjusted_rand_score),
        (F.rand_score, sk.rand_score),
        (F.normalized_mutual_info_score, sk.normalized_mutual_info_score),
        (F.fowlkes_mallows_index, sk.fowlkes_mallows_score),
        (F.homogeneity_score, sk.homogeneity_score),
        (F.completeness_score, sk.completeness_score),
        (F.v_measure_score, sk.v_measure_score),
    ]
    for ours, ref in cases:
        np.testing.assert_allclose(float(ours(pd, td)), ref(tn, pn), rtol=2e-4, err_msg=ours.__name__)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_intrinsic_scores_at_1e6(dtype):
    n, d, k = 1_000_000, 8, 17
    g = torch.Generator().manual_seed(5)
    centers = torch.randn(k, d, generator=g) * 4
    labels = torch.randint(0, k, (n,), generator=g)
    data = (centers[labels] + torch.randn(n, d, generator=g)).to(dtype)
    dd, ld = data.to(DEV), labels.to(DEV)
    xn, ln = data.double().numpy(), labels.numpy()
    rtol = 1e-4 if dtype == torch.float32 else 1e-9
    np.testing.assert_allclose(float(F.calinski_harabasz_score(dd, ld)), sk.calinski_harabasz_score(xn, ln), rtol=rtol)
    np.testing.assert_allclose(float(F.davies_bouldin_score(dd, ld)), sk.davies_bouldin_score(xn, ln), rtol=rtol)
    # Dunn (no sklearn counterpart): against the CPU formulation in fp64
    for p in (2, 1, float("inf")):
        exp = F.dunn_index(data.double(), labels, p)
        np.testing.assert_allclose(float(F.dunn_index(dd, ld, p)), float(exp), rtol=rtol)


def test_dense_labels_match_unique_inverse():
    lab = _labels(300_000, 50, 6, offset=-25, gap=2)
    ids, k = ops.dense_labels(lab.to(DEV))
    uniq, inv = torch.unique(lab, return_inverse=True)
    assert k == uniq.numel() and torch.equal(ids.cpu(), inv)


@pytest.mark.parametrize("n,kp,kt", [(50, 3, 4), (5000, 7, 5), (200_000, 12, 9), (100, 1, 3), (300_000, 300, 300)])
def test_expected_mutual_info_kernel_matches_term_sum(n, kp, kt):
    """csrc/clustering/emi.hip (log-gamma recurrence, one thread per run of terms) against the vectorised fp64 term
    sum on the host (every (i, j, n_ij) term with nine lgamma calls, as the reference)."""
    from torchmetrics_amd.functional import clustering as FC

    g = torch.Generator().manual_seed(n + kp)
    p = torch.randint(0, kp, (n,), generator=g)
    t = torch.randint(0, kt, (n,), generator=g)
    cont = FC._mutual_info_score_update(p, t)
    ref = FC.expected_mutual_info_score(cont, n)
    got = FC.expected_mutual_info_score(cont.cuda(), n)
    assert got.is_cuda
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-6, atol=1e-9)


def test_expected_mutual_info_large_skewed_table():
    """>= 65536 cluster pairs (the tiled emi.hip path) with one giant cluster on each side: the long pair's runs are
    dealt out inside its block; matches the vectorised fp64 term sum."""
    from torchmetrics_amd.functional import clustering as FC

    g = torch.Generator().manual_seed(11)
    n = 100_000
    p = torch.where(torch.rand(n, generator=g) < 0.8, 0, torch.randint(1, 400, (n,), generator=g))
    t = torch.where(torch.rand(n, generator=g) < 0.7, 0, torch.randint(1, 250, (n,), generator=g))
    cont = FC._mutual_info_score_update(p, t)
    assert cont.numel() >= 65536
    ref = FC.expected_mutual_info_score(cont, n)
    got = FC.expected_mutual_info_score(cont.cuda(), n)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-6, atol=1e-9)
