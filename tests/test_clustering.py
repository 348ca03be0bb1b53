"""Clustering metrics vs scikit-learn (reference ``tests/unittests/clustering``)."""
import numpy as np
import pytest
import torch
from sklearn import metrics as skm

from torchmetrics_amd import functional as F
from torchmetrics_amd.clustering import (
    AdjustedMutualInfoScore,
    AdjustedRandScore,
    CalinskiHarabaszScore,
    CompletenessScore,
    DaviesBouldinScore,
    DunnIndex,
    FowlkesMallowsIndex,
    HomogeneityScore,
    MutualInfoScore,
    NormalizedMutualInfoScore,
    RandScore,
    VMeasureScore,
)

_g = torch.Generator().manual_seed(7)
N_BATCH, BS = 4, 64
PREDS = torch.randint(0, 6, (N_BATCH, BS), generator=_g)
TARGET = torch.randint(0, 5, (N_BATCH, BS), generator=_g)
DATA = torch.randn(N_BATCH, BS, 3, generator=_g, dtype=torch.float64)
LABELS = torch.randint(0, 4, (N_BATCH, BS), generator=_g)


def _dunn_ref(data, labels, p=2):
    data, labels = np.asarray(data), np.asarray(labels)
    ks = np.unique(labels)
    cent = np.stack([data[labels == k].mean(0) for k in ks])
    inter = min(np.linalg.norm(cent[i] - cent[j], ord=p) for i in range(len(ks)) for j in range(i + 1, len(ks)))
    intra = max(np.linalg.norm(data[labels == k] - cent[i], ord=p, axis=1).max() for i, k in enumerate(ks))
    return inter / intra


EXTRINSIC = [
    (MutualInfoScore, F.mutual_info_score, skm.mutual_info_score, {}),
    (AdjustedMutualInfoScore, F.adjusted_mutual_info_score, skm.adjusted_mutual_info_score, {}),
    (AdjustedMutualInfoScore, F.adjusted_mutual_info_score, skm.adjusted_mutual_info_score,
     {"average_method": "geometric"}),
    (AdjustedMutualInfoScore, F.adjusted_mutual_info_score, skm.adjusted_mutual_info_score, {"average_method": "max"}),
    (NormalizedMutualInfoScore, F.normalized_mutual_info_score, skm.normalized_mutual_info_score, {}),
    (NormalizedMutualInfoScore, F.normalized_mutual_info_score, skm.normalized_mutual_info_score,
     {"average_method": "min"}),
    (RandScore, F.rand_score, skm.rand_score, {}),
    (AdjustedRandScore, F.adjusted_rand_score, skm.adjusted_rand_score, {}),
    (FowlkesMallowsIndex, F.fowlkes_mallows_index, skm.fowlkes_mallows_score, {}),
    (HomogeneityScore, F.homogeneity_score, skm.homogeneity_score, {}),
    (CompletenessScore, F.completeness_score, skm.completeness_score, {}),
    (VMeasureScore, F.v_measure_score, skm.v_measure_score, {}),
    (VMeasureScore, F.v_measure_score, skm.v_measure_score, {"beta": 2.0}),
]


def _sk(fn, t, p, kw):
    return fn(t.numpy(), p.numpy(), **kw)


@pytest.mark.parametrize(("cls", "fn", "sk", "kw"), EXTRINSIC)
def test_extrinsic_functional(cls, fn, sk, kw):
    for i in range(N_BATCH):
        got = fn(PREDS[i], TARGET[i], **kw)
        assert np.allclose(got.item(), _sk(sk, TARGET[i], PREDS[i], kw), atol=1e-5), (fn.__name__, i)


@pytest.mark.parametrize(("cls", "fn", "sk", "kw"), EXTRINSIC)
def test_extrinsic_module(cls, fn, sk, kw):
    m = cls(**kw)
    for i in range(N_BATCH):
        m.update(PREDS[i], TARGET[i])
    ref = _sk(sk, TARGET.flatten(), PREDS.flatten(), kw)
    assert np.allclose(m.compute().item(), ref, atol=1e-5)


@pytest.mark.parametrize(
    ("cls", "fn", "ref"),
    [
        (CalinskiHarabaszScore, F.calinski_harabasz_score, skm.calinski_harabasz_score),
        (DaviesBouldinScore, F.davies_bouldin_score, skm.davies_bouldin_score),
        (DunnIndex, F.dunn_index, _dunn_ref),
    ],
)
def test_intrinsic(cls, fn, ref):
    for i in range(N_BATCH):
        assert np.allclose(fn(DATA[i], LABELS[i]).item(), ref(DATA[i].numpy(), LABELS[i].numpy()), rtol=1e-6)
    m = cls()
    for i in range(N_BATCH):
        m.update(DATA[i], LABELS[i])
    assert np.allclose(m.compute().item(), ref(DATA.reshape(-1, 3).numpy(), LABELS.flatten().numpy()), rtol=1e-6)


def test_dunn_p1():
    assert np.allclose(F.dunn_index(DATA[0], LABELS[0], p=1).item(), _dunn_ref(DATA[0], LABELS[0], p=1))


def test_edge_cases():
    same = torch.tensor([0, 0, 1, 1, 2])
    assert F.adjusted_rand_score(same, same).item() == 1.0
    assert F.rand_score(same, same).item() == 1.0
    one = torch.zeros(5, dtype=torch.long)
    assert F.mutual_info_score(one, same).item() == 0.0
    assert np.allclose(F.adjusted_mutual_info_score(one, same).item(), skm.adjusted_mutual_info_score(same, one))
    assert np.allclose(F.v_measure_score(one, same).item(), skm.v_measure_score(same, one))
    with pytest.raises(ValueError, match="average_method"):
        F.adjusted_mutual_info_score(same, same, "foo")
    with pytest.raises(ValueError, match="discrete"):
        F.rand_score(same.float(), same)
    with pytest.raises(ValueError, match="Number of detected clusters"):
        F.calinski_harabasz_score(torch.randn(5, 2), one)
    with pytest.raises(ValueError, match="beta"):
        VMeasureScore(beta=0)


def test_contingency_and_pair_matrix():
    p, t = PREDS[0], TARGET[0]
    from sklearn.metrics.cluster import contingency_matrix, pair_confusion_matrix

    from torchmetrics_amd.functional.clustering import (
        calculate_contingency_matrix,
        calculate_pair_cluster_confusion_matrix,
    )
    assert np.array_equal(calculate_contingency_matrix(p, t).numpy(), contingency_matrix(t.numpy(), p.numpy()))
    assert np.array_equal(calculate_pair_cluster_confusion_matrix(p, t).numpy(),
                          pair_confusion_matrix(p.numpy(), t.numpy()))


@pytest.mark.gpu
@pytest.mark.parametrize(("cls", "fn", "sk", "kw"), EXTRINSIC)
def test_extrinsic_gpu(cls, fn, sk, kw):
    m = cls(**kw).cuda()
    for i in range(N_BATCH):
        m.update(PREDS[i].cuda(), TARGET[i].cuda())
    assert np.allclose(m.compute().item(), _sk(sk, TARGET.flatten(), PREDS.flatten(), kw), atol=1e-5)


@pytest.mark.gpu
def test_intrinsic_gpu():
    for cls, ref in ((CalinskiHarabaszScore, skm.calinski_harabasz_score),
                     (DaviesBouldinScore, skm.davies_bouldin_score), (DunnIndex, _dunn_ref)):
        m = cls().cuda()
        for i in range(N_BATCH):
            m.update(DATA[i].cuda(), LABELS[i].cuda())
        assert np.allclose(m.compute().item(), ref(DATA.reshape(-1, 3).numpy(), LABELS.flatten().numpy()), rtol=1e-6)
