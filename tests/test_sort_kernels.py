"""Sorted-curve kernel family (``csrc/sort/clf_curve.hip``) against independent oracles.

sklearn (``roc_auc_score``, ``average_precision_score``, ``roc_curve`` thresholds, label-ranking metrics) and
``scipy.stats.rankdata`` are the oracles; every case runs on the CPU contract (``ops._cpu.clf_curve``) and, with the
``gpu`` marker, on the HIP kernels -- including 10^7-sample columns, heavy ties, bf16 / fp16 / fp64 scores, ignored
targets and sample weights.
"""
import numpy as np
import pytest
import torch
from scipy.stats import rankdata
from sklearn import metrics as skm

from torchmetrics_amd import ops
from torchmetrics_amd.functional.classification import _sorted

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _stats(p, t, tmode, dev, **kw):
    return _sorted.column_stats(p.to(dev), t.to(dev), tmode, **kw)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("levels", [0, 7])  # 0: continuous scores; 7: heavy ties
def test_binary_auroc_ap_vs_sklearn(device, dtype, levels):
    g = torch.Generator().manual_seed(1)
    n = 5000
    p = torch.rand(n, generator=g)
    if levels:
        p = (p * levels).floor() / levels
    p = p.to(dtype)
    t = torch.randint(0, 2, (n,), generator=g)
    st = _stats(p, t, ops.CLF_T_BINARY, device)[0].cpu()
    pn, tn = p.double().numpy(), t.numpy()
    np.testing.assert_allclose(float(_sorted.auroc_from_stats(st)[0]), skm.roc_auc_score(tn, pn), rtol=1e-6)
    np.testing.assert_allclose(float(_sorted.ap_from_stats(st)[0]), skm.average_precision_score(tn, pn), rtol=1e-6)
    assert int(st[0, _sorted.NRUNS]) == len(np.unique(pn))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("ignore", [None, -1])
def test_multiclass_columns_vs_sklearn(device, ignore):
    g = torch.Generator().manual_seed(2)
    m, c = 3000, 7
    p = torch.randn(m, c, generator=g).softmax(-1).round(decimals=2)
    t = torch.randint(0, c, (m,), generator=g)
    if ignore is not None:
        t[::5] = ignore
    st = _stats(p, t, ops.CLF_T_OVR, device, ignore_index=ignore)[0].cpu()
    keep = (t != ignore).numpy() if ignore is not None else np.ones(m, bool)
    auc, ap = _sorted.auroc_from_stats(st), _sorted.ap_from_stats(st)
    for k in range(c):
        y = (t.numpy()[keep] == k)
        s = p[:, k].double().numpy()[keep]
        np.testing.assert_allclose(float(auc[k]), skm.roc_auc_score(y, s), rtol=1e-6)
        np.testing.assert_allclose(float(ap[k]), skm.average_precision_score(y, s), rtol=1e-6)
        assert float(st[k, _sorted.P]) == y.sum() and float(st[k, _sorted.N]) == (~y).sum()


@pytest.mark.parametrize("device", DEVICES)
def test_multilabel_columns_with_ignore_and_curves(device):
    g = torch.Generator().manual_seed(3)
    m, l = 2000, 5
    p = torch.rand(m, l, generator=g).round(decimals=2)
    t = torch.randint(0, 2, (m, l), generator=g)
    t[torch.rand(m, l, generator=g) < 0.1] = -1
    out = _stats(p, t, ops.CLF_T_ELEM, device, ignore_index=-1, emit=ops.EMIT_CURVE)
    fps, tps, thr, host = _sorted.split_curves(out, p.dtype)
    for k in range(l):
        keep = (t[:, k] != -1).numpy()
        y, s = t[:, k].numpy()[keep], p[:, k].numpy()[keep]
        sk_fps, sk_tps, sk_thr = skm._ranking._binary_clf_curve(y, s)
        np.testing.assert_allclose(fps[k].cpu().numpy(), sk_fps)
        np.testing.assert_allclose(tps[k].cpu().numpy(), sk_tps)
        np.testing.assert_allclose(thr[k].cpu().numpy(), sk_thr, rtol=1e-7)


@pytest.mark.parametrize("device", DEVICES)
def test_weighted_binary_curve_vs_sklearn(device):
    g = torch.Generator().manual_seed(4)
    n = 1000
    p = (torch.rand(n, generator=g) * 50).floor() / 50
    t = torch.randint(0, 2, (n,), generator=g)
    w = torch.rand(n, generator=g, dtype=torch.float64)
    out = _stats(p, t, ops.CLF_T_BINARY, device, weights=w.to(device), emit=ops.EMIT_CURVE)
    fps, tps, thr, _ = _sorted.split_curves(out, p.dtype)
    sk_fps, sk_tps, sk_thr = skm._ranking._binary_clf_curve(t.numpy(), p.numpy(), sample_weight=w.numpy())
    np.testing.assert_allclose(fps[0].cpu().numpy(), sk_fps, rtol=1e-5)
    np.testing.assert_allclose(tps[0].cpu().numpy(), sk_tps, rtol=1e-5)
    np.testing.assert_allclose(thr[0].cpu().numpy(), sk_thr)
    np.testing.assert_allclose(float(out[0][0, _sorted.AREA] / (out[0][0, 0] * out[0][0, 1])),
                               skm.roc_auc_score(t.numpy(), p.numpy(), sample_weight=w.numpy()), rtol=1e-6)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_average_ranks_vs_scipy(device, dtype):
    g = torch.Generator().manual_seed(5)
    m, c = 4000, 3
    x = (torch.randn(m, c, generator=g) * 4).round().to(dtype)
    out = _sorted.column_stats(x.to(device), torch.zeros(m, dtype=torch.long, device=device), ops.CLF_T_BINARY,
                               emit=ops.EMIT_RANKS)
    ranks = out[4].cpu().view(c, m)
    for k in range(c):
        np.testing.assert_allclose(ranks[k].numpy(), rankdata(-x[:, k].double().numpy()))


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("shape", [(300, 6), (40, 1500)])
def test_label_ranking_rows_vs_sklearn(device, shape):
    g = torch.Generator().manual_seed(6)
    n, l = shape
    s = torch.rand(n, l, generator=g).round(decimals=1)
    y = torch.randint(0, 2, (n, l), generator=g)
    st = _sorted.row_stats(s.to(device), y.to(device)).cpu()
    p = st[:, 0]
    lrap = torch.where((p > 0) & (p < l), st[:, _sorted.AP] / p.clamp(min=1), torch.ones_like(p)).mean()
    np.testing.assert_allclose(float(lrap), skm.label_ranking_average_precision_score(y.numpy(), s.numpy()), rtol=1e-9)
    np.testing.assert_allclose(float(st[:, _sorted.COV].mean()), skm.coverage_error(y.numpy(), s.numpy()), rtol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [10**6, 10**7])
def test_binary_auroc_large_n_gpu(n):
    g = torch.Generator(device="cuda").manual_seed(7)
    p = torch.rand(n, device="cuda", generator=g)
    t = (torch.rand(n, device="cuda", generator=g) < p).long()  # informative scores
    st = _sorted.column_stats(p, t, ops.CLF_T_BINARY)[0].cpu()
    pn, tn = p.cpu().double().numpy(), t.cpu().numpy()
    np.testing.assert_allclose(float(_sorted.auroc_from_stats(st)[0]), skm.roc_auc_score(tn, pn), rtol=1e-6)
    np.testing.assert_allclose(float(_sorted.ap_from_stats(st)[0]), skm.average_precision_score(tn, pn), rtol=1e-6)


@pytest.mark.gpu
def test_multiclass_many_columns_gpu_matches_cpu_contract():
    g = torch.Generator().manual_seed(8)
    m, c = 20000, 100
    p = torch.randn(m, c, generator=g).softmax(-1).to(torch.bfloat16)
    t = torch.randint(0, c, (m,), generator=g)
    gpu = _sorted.column_stats(p.cuda(), t.cuda(), ops.CLF_T_OVR, emit=ops.EMIT_CURVE)
    cpu = _sorted.column_stats(p, t, ops.CLF_T_OVR, emit=ops.EMIT_CURVE)
    torch.testing.assert_close(gpu[0].cpu(), cpu[0], rtol=1e-9, atol=1e-6)
    n = int(cpu[0][:, _sorted.NRUNS].max())
    for a, b in zip(gpu[1:4], cpu[1:4]):
        mask = torch.arange(m).unsqueeze(0) < cpu[0][:, _sorted.NRUNS].unsqueeze(1)
        torch.testing.assert_close(a.cpu()[mask], b[mask])
    assert n > 0
