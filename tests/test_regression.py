"""Regression metrics vs scikit-learn / scipy oracles (reference test model: ``T/regression``)."""
from functools import partial

import numpy as np
import pytest
import torch
from scipy import stats
from sklearn import metrics as skm

import torchmetrics_amd as tm
import torchmetrics_amd.functional as F
from tests.helpers import assert_close, run_class_test, run_ddp_class_test, run_functional_test

NB, BS = 4, 32
DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _np(x):
    return x.detach().cpu().double().numpy()


def _inputs(k=1, positive=False):
    shape = (NB, BS) if k == 1 else (NB, BS, k)
    p, t = torch.rand(shape), torch.rand(shape)
    if not positive:
        p, t = p * 4 - 2, t * 4 - 2
    return p, t


def _ref(name, preds, target, **kw):
    p, t = _np(preds), _np(target)
    if name == "mse":
        v = skm.mean_squared_error(t, p, multioutput="raw_values" if p.ndim == 2 else "uniform_average")
        return v if kw.get("squared", True) else np.sqrt(v)
    if name == "mae":
        return skm.mean_absolute_error(t.reshape(-1), p.reshape(-1))
    if name == "mape":
        return np.mean(np.abs(p - t) / np.maximum(np.abs(t), 1.17e-06))
    if name == "smape":
        return np.mean(2 * np.abs(p - t) / np.maximum(np.abs(t) + np.abs(p), 1.17e-06))
    if name == "wmape":
        return np.abs(p - t).sum() / np.abs(t).sum()
    if name == "msle":
        return skm.mean_squared_log_error(t, p)
    if name == "logcosh":
        return np.mean(np.log(np.cosh(p - t)), axis=0)
    if name == "r2":
        return skm.r2_score(t, p, multioutput=kw.get("multioutput", "uniform_average"))
    if name == "ev":
        return skm.explained_variance_score(t, p, multioutput=kw.get("multioutput", "uniform_average"))
    if name == "pearson":
        if p.ndim == 2:
            return np.array([stats.pearsonr(t[:, i], p[:, i])[0] for i in range(p.shape[1])])
        return stats.pearsonr(t, p)[0]
    if name == "spearman":
        return stats.spearmanr(t, p)[0]
    if name == "kendall":
        return stats.kendalltau(p, t)[0]
    if name == "minkowski":
        return np.sum(np.abs(p - t) ** kw["p"]) ** (1 / kw["p"])
    if name == "tweedie0":
        return skm.mean_tweedie_deviance(t, p, power=0.0)
    if name == "tweedie15":
        return skm.mean_tweedie_deviance(t, p, power=1.5)
    if name == "concordance":
        mx, my = p.mean(0), t.mean(0)
        vx, vy = p.var(0, ddof=1), t.var(0, ddof=1)
        cov = ((p - mx) * (t - my)).sum(0) / (p.shape[0] - 1)
        return 2 * cov / (vx + vy + (mx - my) ** 2)
    if name == "rse":
        return np.sum((t - p) ** 2) / np.sum((t - t.mean()) ** 2)
    raise ValueError(name)


CASES = [
    ("mse", tm.MeanSquaredError, F.mean_squared_error, {}, False, 1),
    ("mse", tm.MeanSquaredError, F.mean_squared_error, {"squared": False}, False, 1),
    ("mae", tm.MeanAbsoluteError, F.mean_absolute_error, {}, False, 1),
    ("mape", tm.MeanAbsolutePercentageError, F.mean_absolute_percentage_error, {}, False, 1),
    ("smape", tm.SymmetricMeanAbsolutePercentageError, F.symmetric_mean_absolute_percentage_error, {}, False, 1),
    ("wmape", tm.WeightedMeanAbsolutePercentageError, F.weighted_mean_absolute_percentage_error, {}, False, 1),
    ("msle", tm.MeanSquaredLogError, F.mean_squared_log_error, {}, True, 1),
    ("logcosh", tm.LogCoshError, F.log_cosh_error, {}, False, 1),
    ("r2", tm.R2Score, F.r2_score, {}, False, 1),
    ("ev", tm.ExplainedVariance, F.explained_variance, {}, False, 1),
    ("pearson", tm.PearsonCorrCoef, F.pearson_corrcoef, {}, False, 1),
    ("concordance", tm.ConcordanceCorrCoef, F.concordance_corrcoef, {}, False, 1),
    ("spearman", tm.SpearmanCorrCoef, F.spearman_corrcoef, {}, False, 1),
    ("kendall", tm.KendallRankCorrCoef, F.kendall_rank_corrcoef, {}, False, 1),
    ("minkowski", tm.MinkowskiDistance, F.minkowski_distance, {"p": 3}, False, 1),
    ("tweedie0", tm.TweedieDevianceScore, partial(F.tweedie_deviance_score, power=0.0), {"power": 0.0}, False, 1),
    ("tweedie15", tm.TweedieDevianceScore, partial(F.tweedie_deviance_score, power=1.5), {"power": 1.5}, True, 1),
    ("rse", tm.RelativeSquaredError, F.relative_squared_error, {}, False, 1),
]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name,cls,fn,args,positive,k", CASES)
def test_regression(device, name, cls, fn, args, positive, k):
    p, t = _inputs(k, positive)
    ref_kw = {kk: v for kk, v in args.items() if kk in ("squared", "p")}
    ref = partial(_ref, name, **ref_kw)
    fn_args = {kk: v for kk, v in args.items() if kk in ("squared", "p")}
    run_class_test(p, t, cls, ref, metric_args=args, device=device, atol=1e-4)
    run_functional_test(p, t, partial(fn, **fn_args), ref, device=device, atol=1e-4)


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name,cls,extra", [
    ("mse", tm.MeanSquaredError, {"num_outputs": 3}),
    ("r2", tm.R2Score, {"num_outputs": 3, "multioutput": "raw_values"}),
    ("pearson", tm.PearsonCorrCoef, {"num_outputs": 3}),
    ("logcosh", tm.LogCoshError, {"num_outputs": 3}),
])
def test_multioutput(device, name, cls, extra):
    p, t = _inputs(3)
    ref = partial(_ref, name, **({"multioutput": extra["multioutput"]} if "multioutput" in extra else {}))
    run_class_test(p, t, cls, ref, metric_args=extra, device=device, atol=1e-4)


def test_kendall_variants_and_ttest():
    p, t = torch.randint(0, 5, (60,)).float(), torch.randint(0, 5, (60,)).float()
    for v in ("b", "c"):
        tau = F.kendall_rank_corrcoef(p, t, variant=v)
        ref = stats.kendalltau(_np(p), _np(t), variant=v)[0]
        assert_close(tau, ref, atol=1e-5)
    tau, pv = F.kendall_rank_corrcoef(p, t, variant="b", t_test=True)
    assert_close(pv, stats.kendalltau(_np(p), _np(t), variant="b", method="asymptotic")[1], atol=1e-3)


def test_cosine_kl_csi():
    p, t = torch.randn(10, 6), torch.randn(10, 6)
    sk = np.array([np.dot(a, b) / np.linalg.norm(a) / np.linalg.norm(b) for a, b in zip(_np(p), _np(t))])
    assert_close(F.cosine_similarity(p, t, "none"), sk, atol=1e-5)
    m = tm.CosineSimilarity(reduction="mean")
    m.update(p, t)
    assert_close(m.compute(), sk.mean(), atol=1e-5)
    a, b = torch.rand(8, 5), torch.rand(8, 5)
    an, bn = _np(a) / _np(a).sum(1, keepdims=True), _np(b) / _np(b).sum(1, keepdims=True)
    assert_close(F.kl_divergence(a, b), np.mean([stats.entropy(x, y) for x, y in zip(an, bn)]), atol=1e-5)
    pr, tg = torch.rand(5, 4, 4), torch.rand(5, 4, 4)
    h = ((pr >= 0.5) & (tg >= 0.5)).sum()
    mi = ((pr < 0.5) & (tg >= 0.5)).sum()
    fa = ((pr >= 0.5) & (tg < 0.5)).sum()
    assert_close(F.critical_success_index(pr, tg, 0.5), h / (h + mi + fa))


def test_regression_grad_flows():
    p = torch.randn(20, requires_grad=True)
    t = torch.randn(20)
    v = F.mean_squared_error(p, t)
    v.backward()
    assert_close(p.grad, 2 * (p - t).detach() / 20, atol=1e-6)


@pytest.mark.ddp
@pytest.mark.parametrize("name,cls", [("pearson", tm.PearsonCorrCoef), ("mse", tm.MeanSquaredError),
                                      ("spearman", tm.SpearmanCorrCoef), ("r2", tm.R2Score)])
def test_regression_ddp(name, cls):
    p, t = _inputs()
    run_ddp_class_test(p, t, cls, partial(_ref, name), atol=1e-4)


def test_moments_plan_merging_on_cpu(monkeypatch):
    """The collection-level merge of streaming regression requests (ops.run_moments_plans) gives the same values as
    separate updates; forced on CPU tensors so the merge logic (incl. the Pearson-fold / unshifted-sum conflict)
    is covered without a GPU."""
    import torchmetrics_amd as tm
    from torchmetrics_amd import ops
    from torchmetrics_amd import regression as R

    monkeypatch.setattr(ops.MomentsPlan, "deferrable", lambda self: True)
    calls = []
    orig = ops.run_moments_plans
    monkeypatch.setattr(ops, "run_moments_plans", lambda plans, merged_out=None: calls.append(orig(plans, merged_out)))

    def members():
        return {"mse": R.MeanSquaredError(), "r2": R.R2Score(), "pearson": R.PearsonCorrCoef(),
                "concordance": R.ConcordanceCorrCoef(), "ev": R.ExplainedVariance(), "mae": R.MeanAbsoluteError(),
                "mape": R.MeanAbsolutePercentageError(), "mink": R.MinkowskiDistance(p=3.0)}

    coll = tm.MetricCollection(members(), compute_groups=True)
    ref = members()
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        x = torch.randn(500, generator=g) + 2
        y = x + 0.5 * torch.randn(500, generator=g)
        coll.update(x, y)
        for m in ref.values():
            m.update(x, y)
    out = coll.compute()
    for name, m in ref.items():
        torch.testing.assert_close(out[name], m.compute())
    # first update runs every member (group detection); later ones are merged: pearson fold / centred sums /
    # Minkowski power -> 3 kernel calls for 8 metrics
    assert calls and all(c == 3 for c in calls)


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 65, 1000])
@pytest.mark.parametrize("ties", [False, True])
def test_kendall_pair_counts_nlogn_matches_allpairs(n, ties):
    from torchmetrics_amd.functional.regression.correlation import _pair_counts, _pair_counts_allpairs

    g = torch.Generator().manual_seed(n + ties)
    if ties:
        x = torch.randint(0, 5, (n, 3), generator=g).float()
        y = torch.randint(0, 4, (n, 3), generator=g).float()
    else:
        x, y = torch.randn(n, 3, generator=g), torch.randn(n, 3, generator=g)
    c1, d1 = _pair_counts(x, y)
    c2, d2 = _pair_counts_allpairs(x, y)
    assert torch.equal(c1, c2) and torch.equal(d1, d2)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,k", [(8192, 1), (20000, 1), (8192, 2), (6000, 3), (16384, 4)])
def test_moments_mid_size_last_block_fold(rows, k):
    """csrc/regression/moments.hip: mid-size batches (a few blocks of partials) are folded by the last block to finish
    (a per-stream ticket, re-armed by that block) -- repeated updates on one stream against the CPU path."""
    g = torch.Generator().manual_seed(rows + k)
    shape = (rows,) if k == 1 else (rows, k)
    kw = {} if k == 1 else {"num_outputs": k}
    multi = {"multioutput": "raw_values"} if k > 1 else {}
    makers = [lambda: tm.MeanSquaredError(**kw), lambda: tm.MeanAbsoluteError(),
              lambda: tm.R2Score(**kw, **multi), lambda: tm.PearsonCorrCoef(**kw), lambda: tm.ExplainedVariance(**multi)]
    for make in makers:
        gpu, cpu = make().cuda(), make()
        for _ in range(5):
            p, t = torch.randn(shape, generator=g), torch.randn(shape, generator=g)
            gpu.update(p.cuda(), (p + t).cuda())
            cpu.update(p, p + t)
        torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("total", [1024, 16384, 65536])
def test_moments_wave_column_sums(k, total):
    """csrc/common/tm_common.h wave_colsum_f64: per-column wave sums in VALU (row_ror DPP for offsets 1..8, permlane16 /
    permlane32 swaps for 16 / 32) for every power-of-two column count dividing the wave, through the single-block
    (<= 8192 values) and the multi-block hand-off (> 8192) moments kernels -- against the CPU metrics."""
    rows = total // k
    g = torch.Generator().manual_seed(total + k)
    shape = (rows,) if k == 1 else (rows, k)
    kw = {} if k == 1 else {"num_outputs": k}
    multi = {"multioutput": "raw_values"} if k > 1 else {}
    makers = [lambda: tm.MeanSquaredError(**kw), lambda: tm.R2Score(**kw, **multi), lambda: tm.PearsonCorrCoef(**kw)]
    for make in makers:
        gpu, cpu = make().cuda(), make()
        for _ in range(3):
            p, t = torch.randn(shape, generator=g), torch.randn(shape, generator=g)
            gpu.update(p.cuda(), (p + t).cuda())
            cpu.update(p, p + t)
        torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)
