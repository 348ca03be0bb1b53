"""Numerics of the HIP kernels vs the CPU (ATen) implementation of the same op contract.

Every case runs the GPU op and the CPU op on identical inputs and requires identical integer results.
"""
import warnings

import pytest
import torch

from torchmetrics_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _flag(dev):
    return torch.zeros(1, dtype=torch.int32, device=dev)


def _mc(preds, target, C, ignore, mode, samplewise, dev):
    N = target.shape[0]
    if mode == ops.MC_CONFMAT:
        out = torch.zeros(C * C, dtype=torch.int64, device=dev)
    else:
        out = torch.zeros((N if samplewise else 1) * (3 * C + 1), dtype=torch.int64, device=dev)
    flag = _flag(dev)
    ops.mc_update(preds.to(dev), target.to(dev), out, flag, C, ignore, mode, samplewise)
    return out.cpu(), int(flag.item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(257, 5), (1000, 64), (333, 1000), (64, 37), (8, 6, 7), (4, 130, 9), (70001, 10),
                                   (5000, 16), (3000, 31)])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("ignore", [None, 0, -1])
def test_multiclass_argmax(dtype, shape, mode, ignore):
    C = shape[1]
    preds = torch.randn(*shape).to(dtype)
    target = torch.randint(0, C, (shape[0], *shape[2:]))
    if ignore is not None:
        target[::7] = ignore
    g, fg = _mc(preds, target, C, ignore, mode, False, DEV)
    c, fc = _mc(preds, target, C, ignore, mode, False, "cpu")
    assert torch.equal(g, c)
    assert fg == fc == 0


@pytest.mark.parametrize("K", [1, 3])
@pytest.mark.parametrize("samplewise", [False, True])
def test_multiclass_labels(K, samplewise):
    C, N, X = 7, 50, 4
    preds = torch.stack([torch.randperm(C)[:K] for _ in range(N * X)]).view(N, X, K).permute(0, 2, 1).contiguous()
    target = torch.randint(0, C, (N, X))
    g, _ = _mc(preds, target, C, None, ops.MC_STATS, samplewise, DEV)
    c, _ = _mc(preds, target, C, None, ops.MC_STATS, samplewise, "cpu")
    assert torch.equal(g, c)


def test_multiclass_argmax_ties_and_nan():
    preds = torch.zeros(128, 40)
    preds[:, 3] = 1.0
    preds[:, 17] = 1.0  # tie -> first index
    preds[5, 30] = float("nan")  # NaN wins like torch.argmax
    target = torch.randint(0, 40, (128,))
    g, _ = _mc(preds, target, 40, None, ops.MC_CONFMAT, False, DEV)
    c, _ = _mc(preds, target, 40, None, ops.MC_CONFMAT, False, "cpu")
    assert torch.equal(g, c)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [512, 1000, 1024, 1536, 2048])
def test_multiclass_argmax_ord16_edge_rows(dtype, C):
    """The packed-ordinal argmax kernel (16-bit rows of >= 1 KiB) on the rows its shortcut must hand to the float
    compare: +NaN / -NaN (several, different payloads), -0 vs +0 maxima, +-inf, all-equal rows, all-negative rows."""
    N = 20000  # > one row per wave of the persistent grid: exercises the cross-row prefetch
    g = torch.Generator().manual_seed(C)
    preds = torch.randn(N, C, generator=g).to(dtype)
    bits = preds.view(torch.int16)
    nan_pos, nan_neg = (0x7FC1, -0x3F) if dtype == torch.bfloat16 else (0x7E01, -0x1FF)  # -0x3F == 0xFFC1
    for r in range(0, 64):
        bits[r, (r * 37) % C] = nan_pos if r & 1 else nan_neg
        bits[r, (r * 11) % C] = nan_neg if r & 2 else nan_pos + 2
    preds[64:96] = -torch.rand(32, C, generator=g).to(dtype) - 1  # all negative, ties unlikely
    preds[96:128] = 0.0
    preds[96:112, 5] = -0.0
    preds[112:128] = -torch.rand(16, C, generator=g).to(dtype)
    preds[112:128, C - 1] = 0.0
    preds[112:128, 7] = -0.0
    preds[128:160] = float("inf")
    preds[160:192] = float("-inf")
    preds[192:224] = 1.0
    preds[224:256, C // 2] = float("inf")
    preds[224:256, C // 3] = float("inf")
    target = torch.randint(0, C, (N,), generator=g)
    target[::13] = -100
    gpu, fg = _mc(preds, target, C, -100, ops.MC_CONFMAT, False, DEV)
    ref = torch.zeros(C * C, dtype=torch.int64)
    keep = target != -100
    ref += torch.bincount(target[keep] * C + preds.float().argmax(1)[keep], minlength=C * C)
    assert torch.equal(gpu, ref)
    assert fg == 0


def test_multiclass_flags_out_of_range():
    preds = torch.randn(100, 5)
    target = torch.randint(0, 5, (100,))
    target[3] = 9
    g, fg = _mc(preds, target, 5, None, ops.MC_CONFMAT, False, DEV)
    c, fc = _mc(preds, target, 5, None, ops.MC_CONFMAT, False, "cpu")
    assert torch.equal(g, c)
    assert fg == fc != 0


def _bin(preds, target, L, thr, ignore, samplewise, dev, prob_check_all=True):
    N = preds.shape[0]
    G = N * L if samplewise else L
    ws = torch.zeros(G * 7, dtype=torch.int64, device=dev)
    np_ = torch.zeros(1, dtype=torch.int32, device=dev)
    flag = _flag(dev)
    ops.bin_update(preds.to(dev), target.to(dev), ws, flag, np_, L, thr, ignore, samplewise, prob_check_all)
    outs = [torch.zeros(G, dtype=torch.int64, device=dev) for _ in range(4)]
    ops.bin_stats_finalize(ws, np_, True, *outs)
    return torch.stack([o.cpu() for o in outs]), int(flag.item())


@pytest.mark.parametrize("kind", ["prob", "logit", "int"])
@pytest.mark.parametrize("shape,L", [((1000,), 1), ((64, 9), 9), ((16, 3, 2000), 3), ((8, 2, 5), 2),
                                     ((300000,), 1), ((3000, 100), 100), ((700, 1000), 1000), ((40, 7, 13), 7),
                                     ((500, 1001), 1001)])
@pytest.mark.parametrize("samplewise", [False, True])
@pytest.mark.parametrize("ignore", [None, -1])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_binary_like(kind, shape, L, samplewise, ignore, dtype):
    if kind == "prob":
        preds = torch.rand(*shape).to(dtype)
    elif kind == "logit":
        preds = (torch.randn(*shape) * 3).to(dtype)
    else:
        preds = torch.randint(0, 2, shape)
    target = torch.randint(0, 2, shape)
    if ignore is not None:
        target.view(-1)[::5] = ignore
    g, fg = _bin(preds, target, L, 0.5, ignore, samplewise, DEV)
    c, fc = _bin(preds, target, L, 0.5, ignore, samplewise, "cpu")
    assert torch.equal(g, c)
    assert fg == fc


def test_binary_confmat_prob_check_excludes_ignored():
    preds = torch.rand(300)
    target = torch.randint(0, 2, (300,))
    preds[0] = 5.0  # out of [0,1] but ignored -> stays probability interpretation
    target[0] = -1
    dev_res = []
    for dev in (DEV, "cpu"):
        ws = torch.zeros(7, dtype=torch.int64, device=dev)
        np_ = torch.zeros(1, dtype=torch.int32, device=dev)
        cm = torch.zeros(2, 2, dtype=torch.int64, device=dev)
        ops.bin_update(preds.to(dev), target.to(dev), ws, _flag(dev), np_, 1, 0.5, -1, False, False)
        ops.bin_confmat_finalize(ws, np_, cm)
        dev_res.append(cm.cpu())
    assert torch.equal(dev_res[0], dev_res[1])


@pytest.mark.parametrize("n,bins", [(10000, 37), (100000, 20000), (5, 3)])
def test_histogram(n, bins):
    x = torch.randint(0, bins, (n,))
    assert torch.equal(ops.histogram(x.to(DEV), bins).cpu(), torch.bincount(x, minlength=bins))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C", [3, 10, 64, 100, 1000])
@pytest.mark.parametrize("kind", ["logits", "probs"])
def test_calibration_fused_update_matches_cpu(dtype, C, kind):
    """Fused top-label update (csrc/classification/calibration.hip) vs the CPU path of the same metric, over
    several updates (exercises the double-buffered softmax decision word)."""
    import torchmetrics_amd as tm

    g = torch.Generator().manual_seed(C)
    gpu = tm.MulticlassCalibrationError(num_classes=C, n_bins=15).to(DEV)
    cpu = tm.MulticlassCalibrationError(num_classes=C, n_bins=15)
    for step in range(4):
        x = torch.randn(777, C, generator=g)
        if kind == "probs" or step == 2:  # mixed batches: decision is per update
            x = x.softmax(1)
        x = x.to(dtype)
        y = torch.randint(0, C, (777,), generator=g)
        gpu.update(x.to(DEV), y.to(DEV))
        cpu.update(x, y)
    for a, b in zip(gpu.confidences, cpu.confidences):
        # one unit in the last place of the input dtype (CPU and GPU expf may round a softmax value differently)
        atol = {torch.float32: 1e-6, torch.bfloat16: 4e-3, torch.float16: 1e-3}[dtype]
        torch.testing.assert_close(a.cpu(), b, rtol=0, atol=atol)
    for a, b in zip(gpu.accuracies, cpu.accuracies):
        assert torch.equal(a.cpu(), b)
    torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)


def test_calibration_fused_flags_target_range():
    import torchmetrics_amd as tm

    m = tm.MulticlassCalibrationError(num_classes=5).to(DEV)
    y = torch.randint(0, 5, (64,))
    y[7] = 9
    m.update(torch.randn(64, 5, device=DEV), y.to(DEV))
    with pytest.raises(RuntimeError):
        m.compute()


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("n", [1000, 20000])
def test_collection_merged_moments_matches_individual(k, n):
    """A MetricCollection merges its streaming regression members' kernel requests into one pass
    (ops.run_moments_plans); results must equal each metric updated alone on the CPU."""
    import torchmetrics_amd as tm
    from torchmetrics_amd import regression as R

    def members():
        common = {
            "mse": R.MeanSquaredError(num_outputs=k), "r2": R.R2Score(num_outputs=k),
            "pearson": R.PearsonCorrCoef(num_outputs=k), "concordance": R.ConcordanceCorrCoef(num_outputs=k),
            "ev": R.ExplainedVariance(),
        }
        if k == 1:
            common.update({"mae": R.MeanAbsoluteError(), "mape": R.MeanAbsolutePercentageError(),
                           "mink": R.MinkowskiDistance(p=3.0), "logcosh": R.LogCoshError(), "smape":
                           R.SymmetricMeanAbsolutePercentageError()})
        return common

    gpu = tm.MetricCollection(members(), compute_groups=True).to(DEV)
    cpu = members()
    g = torch.Generator().manual_seed(n + k)
    for step in range(3):
        x = torch.randn(n, k, generator=g).squeeze(-1) + 2
        y = x + 0.5 * torch.randn(n, k, generator=g).squeeze(-1)
        gpu.update(x.to(DEV), y.to(DEV))
        for m in cpu.values():
            m.update(x, y)
    out = gpu.compute()
    for name, m in cpu.items():
        torch.testing.assert_close(out[name].cpu().float(), m.compute().float(), rtol=2e-4, atol=1e-5)


@pytest.mark.parametrize("task", ["multiclass", "multilabel"])
@pytest.mark.parametrize("metric", ["auroc", "ap"])
@pytest.mark.parametrize("average", ["macro", "weighted", "none"])
@pytest.mark.parametrize("C", [3, 10, 130])
def test_curve_score_fused_matches_cpu(task, metric, average, C):
    """Binned AUROC / AP compute through the fused curve_score kernel vs the CPU op-by-op formulation, including
    classes with no positives (NaN AUROC, nan-aware averages)."""
    import torchmetrics_amd as tm

    g = torch.Generator().manual_seed(C)
    n = 600
    if task == "multiclass":
        preds = torch.randn(n, C, generator=g).softmax(1)
        target = torch.randint(0, max(C - 1, 2), (n,), generator=g)  # last class never appears
        cls = {"auroc": tm.MulticlassAUROC, "ap": tm.MulticlassAveragePrecision}[metric]
        kw = {"num_classes": C}
    else:
        preds = torch.rand(n, C, generator=g)
        target = (torch.rand(n, C, generator=g) > 0.6).long()
        target[:, -1] = 0
        cls = {"auroc": tm.MultilabelAUROC, "ap": tm.MultilabelAveragePrecision}[metric]
        kw = {"num_labels": C}
    gpu = cls(thresholds=50, average=average, **kw).to(DEV)
    cpu = cls(thresholds=50, average=average, **kw)
    gpu.update(preds.to(DEV), target.to(DEV))
    cpu.update(preds, target)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        a, b = gpu.compute().cpu(), cpu.compute()
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, equal_nan=True)


def _confmats(C, g):
    cms = [torch.randint(0, 50, (C, C), generator=g)]
    z = torch.zeros(C, C, dtype=torch.int64)
    z[0, 0] = 7  # a single class seen
    cms.append(z)
    d = torch.diag(torch.randint(1, 9, (C,), generator=g))  # perfect predictions
    cms.append(d)
    e = torch.randint(0, 5, (C, C), generator=g)
    e[C - 1, :] = 0
    e[:, C - 1] = 0  # a class never seen
    cms.append(e)
    return cms


@pytest.mark.parametrize("C", [2, 3, 10, 257])
def test_confmat_reduce_matches_cpu(C):
    """Fused Jaccard / Cohen kappa / MCC (csrc/classification/confmat_reduce.hip) vs the CPU formulations, on
    random, single-class, perfect and missing-class matrices (incl. the degenerate 2x2 MCC cases)."""
    from torchmetrics_amd.functional.classification.cohen_kappa import _cohen_kappa_reduce
    from torchmetrics_amd.functional.classification.jaccard import _jaccard_index_reduce
    from torchmetrics_amd.functional.classification.matthews_corrcoef import _matthews_corrcoef_reduce

    g = torch.Generator().manual_seed(C)
    cms = _confmats(C, g)
    if C == 2:
        cms += [torch.tensor([[5, 0], [0, 0]]), torch.tensor([[0, 0], [0, 5]]), torch.tensor([[0, 3], [0, 0]]),
                torch.tensor([[0, 0], [4, 0]]), torch.tensor([[3, 2], [0, 0]]), torch.tensor([[0, 0], [2, 3]])]
    for cm in cms:
        for avg in ("micro", "macro", "weighted", "none"):
            for ii in (None, 0, C + 3):
                a = _jaccard_index_reduce(cm.to(DEV), avg, ii).cpu()
                b = _jaccard_index_reduce(cm, avg, ii)
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, equal_nan=True)
        for w in (None, "linear", "quadratic"):
            torch.testing.assert_close(_cohen_kappa_reduce(cm.to(DEV), w).cpu(), _cohen_kappa_reduce(cm, w),
                                       rtol=1e-5, atol=1e-6, equal_nan=True)
        torch.testing.assert_close(_matthews_corrcoef_reduce(cm.to(DEV)).cpu().float(),
                                   _matthews_corrcoef_reduce(cm).float(), rtol=1e-5, atol=1e-6, equal_nan=True)


@pytest.mark.parametrize("n_bins", [1, 15, 16, 17, 100])
def test_calibration_bins_matches_cpu(n_bins):
    from torchmetrics_amd.functional.classification.calibration_error import _binning_bucketize

    g = torch.Generator().manual_seed(n_bins)
    conf = torch.rand(100000, generator=g)
    conf[:7] = 1.0  # the last boundary: its own slot, as torch.bucketize(right=True) - 1
    conf[7:9] = 0.0
    acc = (torch.rand(100000, generator=g) > 0.4).float()
    bounds = torch.linspace(0, 1, n_bins + 1)
    ref = _binning_bucketize(conf, acc, bounds)
    got = _binning_bucketize(conf.to(DEV), acc.to(DEV), bounds.to(DEV))
    for a, b in zip(got, ref):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-4, atol=1e-6)


def test_graphed_update_matches_eager():
    """HIP-graph replay of update (utils.graphs.GraphedUpdate) for a metric and two collections equals eager updates;
    list-state metrics are refused; reset + recapture works."""
    import torchmetrics_amd as tm
    from torchmetrics_amd import classification as C
    from torchmetrics_amd import regression as R
    from torchmetrics_amd.utils.graphs import GraphedUpdate

    def cls_coll():
        return tm.MetricCollection({
            "acc": C.MulticlassAccuracy(10), "f1": C.MulticlassF1Score(10), "cm": C.MulticlassConfusionMatrix(10),
            "jacc": C.MulticlassJaccardIndex(10), "mcc": C.MulticlassMatthewsCorrCoef(10),
            "auroc": C.MulticlassAUROC(10, thresholds=50), "ap": C.MulticlassAveragePrecision(10, thresholds=50),
        }, compute_groups=True).to(DEV)

    def reg_coll():
        return tm.MetricCollection({"mse": R.MeanSquaredError(), "mae": R.MeanAbsoluteError(), "r2": R.R2Score(),
                                    "pearson": R.PearsonCorrCoef(), "ev": R.ExplainedVariance()}).to(DEV)

    g = torch.Generator().manual_seed(0)
    batches = [(torch.randn(512, 10, generator=g).to(DEV, torch.bfloat16), torch.randint(0, 10, (512,), generator=g).to(DEV),
                torch.randn(512, generator=g).to(DEV)) for _ in range(5)]
    eager_c, eager_r, eager_m = cls_coll(), reg_coll(), C.MulticlassConfusionMatrix(10).to(DEV)
    graph_c, graph_r, graph_m = cls_coll(), reg_coll(), C.MulticlassConfusionMatrix(10).to(DEV)
    gc = GraphedUpdate(graph_c, batches[0][0], batches[0][1])
    gr = GraphedUpdate(graph_r, batches[0][2], batches[0][2] * 0.5 + 0.1)
    gm = GraphedUpdate(graph_m, batches[0][0], batches[0][1])
    for p, t, x in batches:
        y = x * 0.5 + 0.1 * torch.sin(x)
        eager_c.update(p, t)
        eager_r.update(x, y)
        eager_m.update(p, t)
        gc(p, t)
        gr(x, y)
        gm(p, t)
    a, b = graph_c.compute(), eager_c.compute()
    for k in b:
        torch.testing.assert_close(a[k], b[k])
    a, b = graph_r.compute(), eager_r.compute()
    for k in b:
        torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-6)
    assert torch.equal(graph_m.compute(), eager_m.compute()) and graph_m.update_count == eager_m.update_count == 5
    graph_m.reset()
    gm.recapture()
    gm(batches[0][0], batches[0][1])
    eager_m.reset()
    eager_m.update(batches[0][0], batches[0][1])
    assert torch.equal(graph_m.compute(), eager_m.compute())
    with pytest.raises(ValueError, match="list state"):
        GraphedUpdate(C.MulticlassCalibrationError(10).to(DEV), batches[0][0], batches[0][1])


@pytest.mark.parametrize("n", [64, 4096, 70000])
def test_graphed_update_decides_logits_per_batch(n):
    """The 'scores are not probabilities' decision is per batch under graph replay too: batches that
    alternate between logits and probabilities, replayed from one captured graph and interleaved with eager updates
    of the same metric, equal eager-only updates -- binary / multilabel stat scores, the binary confusion matrix and
    the fused multiclass family (binned AUROC / AP soften logits only)."""
    import torchmetrics_amd as tm
    from torchmetrics_amd import classification as C
    from torchmetrics_amd.utils.graphs import GraphedUpdate

    g = torch.Generator().manual_seed(3)

    def batch(kind, logits):
        if kind == "bin":
            p = torch.randn(n, generator=g) * 3 if logits else torch.rand(n, generator=g)
            return p.to(DEV), torch.randint(0, 2, (n,), generator=g).to(DEV)
        if kind == "ml":
            p = torch.randn(n, 5, generator=g) * 3 if logits else torch.rand(n, 5, generator=g)
            return p.to(DEV), torch.randint(0, 2, (n, 5), generator=g).to(DEV)
        p = torch.randn(n, 6, generator=g) * 3 if logits else torch.softmax(torch.randn(n, 6, generator=g), 1)
        return p.to(DEV, torch.bfloat16), torch.randint(0, 6, (n,), generator=g).to(DEV)

    makers = {
        "bin": lambda: [C.BinaryAccuracy(), C.BinaryF1Score(), C.BinaryConfusionMatrix()],
        "ml": lambda: [C.MultilabelF1Score(5, average="macro"), C.MultilabelAccuracy(5, average=None)],
        "mc": lambda: [tm.MetricCollection({
            "acc": C.MulticlassAccuracy(6), "cm": C.MulticlassConfusionMatrix(6),
            "auroc": C.MulticlassAUROC(6, thresholds=20), "ap": C.MulticlassAveragePrecision(6, thresholds=20)},
            compute_groups=True)],
    }
    pattern = [True, False, False, True, False, True, True, False]
    for kind, make in makers.items():
        eager = [m.to(DEV) for m in make()]
        graphed = [m.to(DEV) for m in make()]
        first = batch(kind, True)
        runners = [GraphedUpdate(m, *first) for m in graphed]
        for i, logits in enumerate(pattern):
            p, t = batch(kind, logits)
            for m in eager:
                m.update(p, t)
            for m, r in zip(graphed, runners):
                if i % 3 == 2:
                    m.update(p, t)  # eager update of the graphed metric between replays
                else:
                    r(p, t)
        for a, b in zip(graphed, eager):
            ra, rb = a.compute(), b.compute()
            if isinstance(rb, dict):
                for k in rb:
                    torch.testing.assert_close(ra[k], rb[k], msg=f"{kind}/{k}")
            else:
                torch.testing.assert_close(ra, rb, msg=kind)


# ------------------------------------------------------------------ fused regression compute (regression_compute.hip)
def _reg_cases():
    g = torch.Generator().manual_seed(7)
    t = torch.randn(500, 4, generator=g)
    p = t + 0.3 * torch.randn(500, 4, generator=g)
    p[:, 1] = t[:, 1]  # perfect column: zero numerator / rss
    t2 = t.clone()
    t2[:, 2] = 1.5  # constant target column: zero denominator / tss
    p2 = p.clone()
    p2[:, 3] = 2.0  # constant prediction column (Pearson low variance)
    return [(p, t), (p, t2), (p2, t2), (p[:, 0], t[:, 0])]


@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("multioutput", ["raw_values", "uniform_average", "variance_weighted"])
def test_fused_ev_r2_compute_matches_cpu(case, dtype, multioutput):
    from torchmetrics_amd.functional.regression.streaming import (
        _explained_variance_compute, _explained_variance_update, _r2_score_compute, _r2_score_update)

    p, t = (x.to(dtype) for x in _reg_cases()[case])
    ev_states = _explained_variance_update(p, t)
    ref = _explained_variance_compute(*ev_states, multioutput)
    got = _explained_variance_compute(*(s.to(DEV) if isinstance(s, torch.Tensor) else s for s in ev_states),
                                      multioutput)
    assert got.shape == ref.shape and got.is_cuda
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-5, atol=1e-6, equal_nan=True)
    r2_states = _r2_score_update(p, t)
    for n in (r2_states[3], torch.tensor(r2_states[3])):
        ref = _r2_score_compute(*r2_states[:3], n, 0, multioutput)
        got = _r2_score_compute(*(s.to(DEV) for s in r2_states[:3]), n.to(DEV) if isinstance(n, torch.Tensor) else n,
                                0, multioutput)
        assert got.shape == ref.shape and got.is_cuda
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-5, atol=1e-6, equal_nan=True)


def test_fused_r2_module_paths():
    from torchmetrics_amd.regression import R2Score

    p, t = _reg_cases()[0]
    for adjusted in (0, 2):
        cpu, gpu = R2Score(num_outputs=4, adjusted=adjusted), R2Score(num_outputs=4, adjusted=adjusted).to(DEV)
        cpu.update(p, t)
        gpu.update(p.to(DEV), t.to(DEV))
        torch.testing.assert_close(gpu.compute().cpu(), cpu.compute(), rtol=1e-5, atol=1e-6)
    one = R2Score().to(DEV)
    one.update(p[:1, 0].to(DEV), t[:1, 0].to(DEV))
    with pytest.raises(ValueError, match="at least two samples"):
        one.compute()


@pytest.mark.parametrize("case", range(4))
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_fused_pearson_concordance_matches_cpu(case, dtype):
    from torchmetrics_amd.regression import ConcordanceCorrCoef, PearsonCorrCoef

    p, t = (x.to(dtype) for x in _reg_cases()[case])
    k = p.shape[1] if p.ndim == 2 else 1
    for cls in (PearsonCorrCoef, ConcordanceCorrCoef):
        cpu, gpu = cls(num_outputs=k), cls(num_outputs=k).to(DEV)
        if dtype == torch.float64:
            cpu, gpu = cpu.double(), gpu.double()
        for lo in range(0, 500, 128):
            cpu.update(p[lo:lo + 128], t[lo:lo + 128])
            gpu.update(p[lo:lo + 128].to(DEV), t[lo:lo + 128].to(DEV))
        with warnings.catch_warnings(record=True) as wc:
            warnings.simplefilter("always")
            ref = cpu.compute()
        with warnings.catch_warnings(record=True) as wg:
            warnings.simplefilter("always")
            got = gpu.compute()
        assert got.shape == ref.shape
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-5, equal_nan=True)
        low = lambda ws: any("variance of predictions or target" in str(w.message) for w in ws)  # noqa: E731
        assert low(wg) == low(wc)


def test_graphed_update_bound_input_ring():
    """bind_inputs=True: one graph per buffer of an input ring reads the buffers in place; refilled buffers give the
    same states as eager updates on the same batches."""
    import torchmetrics_amd as tm
    from torchmetrics_amd import classification as C
    from torchmetrics_amd import regression as R
    from torchmetrics_amd.utils.graphs import GraphedUpdate

    def coll():
        return tm.MetricCollection({"acc": C.MulticlassAccuracy(7), "cm": C.MulticlassConfusionMatrix(7),
                                    "auroc": C.MulticlassAUROC(7, thresholds=20)}, compute_groups=True).to(DEV)

    g = torch.Generator().manual_seed(1)
    ring = [(torch.empty(300, 7, device=DEV), torch.empty(300, dtype=torch.long, device=DEV)) for _ in range(3)]
    for p, t in ring:
        p.copy_(torch.randn(300, 7, generator=g))
        t.copy_(torch.randint(0, 7, (300,), generator=g))
    eager, graphed = coll(), coll()
    reg_e, reg_g = R.MeanSquaredError().to(DEV), R.MeanSquaredError().to(DEV)
    graphs = [GraphedUpdate(graphed, p, t, bind_inputs=True) for p, t in ring]
    rgraphs = [GraphedUpdate(reg_g, p[:, 0].contiguous(), p[:, 1].contiguous(), bind_inputs=True) for p, _ in ring]
    for step in range(7):
        i = step % 3
        p, t = ring[i]
        p.copy_(torch.randn(300, 7, generator=g))  # the producer refills the slot in place
        t.copy_(torch.randint(0, 7, (300,), generator=g))
        eager.update(p, t)
        graphs[i]()  # no arguments: read the bound buffers
        x, y = rgraphs[i]._static
        x.copy_(p[:, 0])
        y.copy_(p[:, 1])
        reg_e.update(x, y)
        rgraphs[i](x, y)  # the bound tensors themselves: no copy
    a, b = graphed.compute(), eager.compute()
    for k in b:
        torch.testing.assert_close(a[k], b[k])
    torch.testing.assert_close(reg_g.compute(), reg_e.compute())
    assert graphed["acc"].update_count == eager["acc"].update_count == 7


@pytest.mark.parametrize("norm", ["l1", "max", "l2"])
@pytest.mark.parametrize("n_bins", [1, 15, 16, 17, 100])
@pytest.mark.parametrize("n", [50000, 2000003])
def test_calibration_error_compute_matches_cpu(norm, n_bins, n):
    from torchmetrics_amd.functional.classification.calibration_error import _ce_compute

    g = torch.Generator().manual_seed(n_bins + len(norm))
    conf = torch.rand(n, generator=g)
    conf[:5] = 1.0
    acc = (torch.rand(n, generator=g) > 0.3).float()
    ref = _ce_compute(conf.double(), acc.double(), n_bins, norm).float()
    for _ in range(2):  # the second call reuses the (self-clearing) bin workspace
        got = _ce_compute(conf.to(DEV), acc.to(DEV), n_bins, norm)
        assert got.shape == ref.shape
        torch.testing.assert_close(got.cpu().float(), ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("C", [3, 10, 32, 33])
@pytest.mark.parametrize("kind", ["logits", "probs"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_multiclass_binned_curve_state_matches_cpu(C, kind, dtype):
    """Small-C multiclass binning (fused two-plane kernel for C <= 32) == the CPU state, incl. ignore_index."""
    from torchmetrics_amd.classification import MulticlassPrecisionRecallCurve

    g = torch.Generator().manual_seed(C)
    x = torch.randn(3000, C, generator=g)
    preds = (x.softmax(-1) if kind == "probs" else x * 3).to(dtype)
    target = torch.randint(0, C, (3000,), generator=g)
    target[::17] = -1
    cpu = MulticlassPrecisionRecallCurve(C, thresholds=37, ignore_index=-1)
    gpu = MulticlassPrecisionRecallCurve(C, thresholds=37, ignore_index=-1).to(DEV)
    for lo in range(0, 3000, 1000):
        cpu.update(preds[lo:lo + 1000], target[lo:lo + 1000])
        gpu.update(preds[lo:lo + 1000].to(DEV), target[lo:lo + 1000].to(DEV))
    assert torch.equal(gpu.confmat.cpu(), cpu.confmat)
