"""``GraphedCompute``: per-step compute() of a collection replayed from one HIP graph.

Checked against a twin collection that takes the eager path on the same batches (values must match exactly: the
same kernels run on the same states), across resets, on a bad batch (must raise the member's own error), and under
a simulated 2-rank job (two processes on one device, arena buckets reduced by the one-shot kernel) against a
single-process CPU collection fed every rank's batches.
"""
import copy

import pytest
import torch

from tests.helpers import run_ddp

pytestmark = pytest.mark.gpu

NC = 7


def _collection(device):
    from torchmetrics_amd import MetricCollection
    from torchmetrics_amd import classification as C
    from torchmetrics_amd import regression as R

    cls = MetricCollection({
        "acc": C.MulticlassAccuracy(NC, average="macro"),
        "prec": C.MulticlassPrecision(NC, average="weighted"),
        "f1": C.MulticlassF1Score(NC, average="micro"),
        "spec": C.MulticlassSpecificity(NC, average="none"),
        "stat": C.MulticlassStatScores(NC, average="macro"),
        "jacc": C.MulticlassJaccardIndex(NC),
        "mcc": C.MulticlassMatthewsCorrCoef(NC),
        "kappa": C.MulticlassCohenKappa(NC),
        "cm": C.MulticlassConfusionMatrix(NC),
        "auroc": C.MulticlassAUROC(NC, thresholds=50),
        "ap": C.MulticlassAveragePrecision(NC, thresholds=50),
        "roc": C.MulticlassROC(NC, thresholds=20),
        "ece": C.MulticlassCalibrationError(NC, n_bins=10),
    }, compute_groups=True).to(device)
    reg = MetricCollection({
        "mse": R.MeanSquaredError(), "mae": R.MeanAbsoluteError(), "r2": R.R2Score(),
        "pearson": R.PearsonCorrCoef(), "ev": R.ExplainedVariance(),
    }, compute_groups=True).to(device)
    return cls, reg


def _batch(seed, n=512, device="cuda"):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(n, NC, generator=g)
    labels = torch.randint(0, NC, (n,), generator=g)
    x = torch.randn(n, generator=g)
    y = x + 0.3 * torch.randn(n, generator=g)
    return logits.to(device), labels.to(device), x.to(device), y.to(device)


def _assert_same(a, b):
    if isinstance(a, dict):
        assert a.keys() == b.keys()
        for k in a:
            _assert_same(a[k], b[k])
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            _assert_same(x, y)
    else:
        torch.testing.assert_close(a.cpu(), b.cpu(), rtol=1e-6, atol=1e-7, equal_nan=True)


def test_graphed_compute_matches_eager_every_step():
    from torchmetrics_amd.utils.graphs import GraphedCompute

    cls, reg = _collection("cuda")
    twin_cls, twin_reg = copy.deepcopy(cls), copy.deepcopy(reg)
    lg, lb, x, y = _batch(0)
    for c, r in ((cls, reg), (twin_cls, twin_reg)):
        c.update(lg, lb)
        r.update(x, y)
    g_cls, g_reg = GraphedCompute(cls), GraphedCompute(reg)
    assert {n for n, _ in g_cls._graphed} >= {"acc", "cm", "auroc", "ap", "mcc"}, g_cls._capture_errors
    assert "ece" in {n for n, _ in g_cls._eager}  # list states stay eager
    assert len(g_reg._eager) == 0, g_reg._capture_errors
    for step in range(1, 6):
        _assert_same(g_cls(), twin_cls.compute())
        _assert_same(g_reg(), twin_reg.compute())
        lg, lb, x, y = _batch(step)
        for c, r in ((cls, reg), (twin_cls, twin_reg)):
            c.update(lg, lb)
            r.update(x, y)
    # reset re-creates the state tensors: the arena packs the live ones, no recapture needed
    for c in (cls, reg, twin_cls, twin_reg):
        c.reset()
    lg, lb, x, y = _batch(99)
    for c, r in ((cls, reg), (twin_cls, twin_reg)):
        c.update(lg, lb)
        r.update(x, y)
    _assert_same(g_cls(), twin_cls.compute())
    _assert_same(g_reg(), twin_reg.compute())


def test_one_graph_for_two_collections():
    from torchmetrics_amd.utils.graphs import GraphedCompute

    cls, reg = _collection("cuda")
    twin_cls, twin_reg = copy.deepcopy(cls), copy.deepcopy(reg)
    for step in range(3):
        lg, lb, x, y = _batch(40 + step)
        for c, r in ((cls, reg), (twin_cls, twin_reg)):
            c.update(lg, lb)
            r.update(x, y)
        if step == 0:
            g = GraphedCompute(cls, reg)
        a, b = g()
        _assert_same(a, twin_cls.compute())
        _assert_same(b, twin_reg.compute())


def test_results_are_not_overwritten_by_the_next_replay():
    from torchmetrics_amd.utils.graphs import GraphedCompute

    cls, _ = _collection("cuda")
    lg, lb, _, _ = _batch(1)
    cls.update(lg, lb)
    g = GraphedCompute(cls)
    first = g()
    kept = first["acc"].clone()
    lg, lb, _, _ = _batch(2)
    cls.update(lg, lb)
    second = g()
    assert torch.equal(first["acc"], kept)
    assert not torch.equal(second["cm"], first["cm"])


def test_bad_batch_raises_from_graphed_compute():
    from torchmetrics_amd.utils.graphs import GraphedCompute

    cls, _ = _collection("cuda")
    lg, lb, _, _ = _batch(3)
    cls.update(lg, lb)
    g = GraphedCompute(cls)
    g()
    lb = lb.clone()
    lb[5] = NC + 3
    cls.update(lg, lb)
    with pytest.raises((ValueError, RuntimeError)):
        g()


# ---------------------------------------------------------------------------------- simulated 2-rank job
def _body_two_rank(rank, world):
    from torchmetrics_amd.parallel import sync
    from torchmetrics_amd.parallel.oneshot import OneShotAllReduce
    from torchmetrics_amd.utils.graphs import GraphedCompute

    torch.cuda.set_device(0)
    comm = OneShotAllReduce(None, allow_shared_device=True)
    assert comm.usable
    sync._is_nccl = lambda group: True
    sync.get_oneshot = lambda group: comm
    try:
        from torchmetrics_amd import MetricCollection
        from torchmetrics_amd import classification as C

        def build(dev, **kw):
            return MetricCollection({
                "acc": C.MulticlassAccuracy(NC, average="macro", **kw),
                "cm": C.MulticlassConfusionMatrix(NC, **kw),
                "kappa": C.MulticlassCohenKappa(NC, **kw),
                "auroc": C.MulticlassAUROC(NC, thresholds=30, **kw),
            }, compute_groups=True).to(dev)

        # every member is graphable, so only the arena buckets travel (through the one-shot kernel)
        coll = build("cuda")
        ref = build("cpu", sync_on_compute=False)  # fed every rank's batches itself
        for step in range(3):
            for r in range(world):
                lg, lb, _, _ = _batch(10 * step + r, device="cpu")
                ref.update(lg, lb)
            lg, lb, _, _ = _batch(10 * step + rank, device="cpu")
            coll.update(lg.cuda(), lb.cuda())
        g = GraphedCompute(coll)
        assert g._world_size == world and len(g._eager) == 0
        out = g()
        exp = ref.compute()
        for k in exp:
            torch.testing.assert_close(out[k].cpu().to(exp[k].dtype), exp[k], rtol=1e-5, atol=1e-6)
        # local states are untouched: a local-only compute still sees one rank's data
        assert int(coll["cm"].confmat.sum()) == 3 * 512
        comm.check()
    finally:
        torch.cuda.synchronize()
        import torch.distributed as dist

        dist.barrier()
        comm.close()


def test_graphed_compute_two_ranks_one_device():
    run_ddp(_body_two_rank)


# ---------------------------------------------------------------------------------- one-launch task kernel
def _stat_scores_ref(tp, fp, tn, fn, average):
    from torchmetrics_amd.functional.classification.stat_scores import _multiclass_stat_scores_compute

    return _multiclass_stat_scores_compute(tp, fp, tn, fn, average)


def test_fused_compute_tasks_match_standalone_kernels():
    """Every reduction recorded by ops.fused_compute and run by compute_tasks equals its standalone kernel."""
    from torchmetrics_amd import ops

    g = torch.Generator().manual_seed(5)
    dev = "cuda"
    calls = []
    for kind in range(6):
        for avg in range(4):
            for ml in (False, True):
                st = [torch.randint(0, 50, (3, 11), generator=g).to(dev) for _ in range(4)]
                calls.append(lambda st=st, kind=kind, avg=avg, ml=ml: ops.stat_reduce(*st, kind, avg, ml, 0.5))
    for c in (2, 5, 40):
        cm = torch.randint(0, 30, (c, c), generator=g).to(dev)
        for kind, avg, w in ((0, "macro", None), (0, "micro", None), (0, "weighted", None), (0, None, None),
                             (1, "macro", None), (1, "macro", "linear"), (1, "macro", "quadratic"), (2, "macro", None)):
            calls.append(lambda cm=cm, kind=kind, avg=avg, w=w: ops.confmat_reduce(cm, kind, avg, 1, w))
    for c in (1, 4, 100):
        state = torch.randint(0, 40, (25, c, 2, 2), generator=g).to(dev)
        for kind in (0, 1):
            for avg in (None, "macro", "weighted"):
                calls.append(lambda s=state, kind=kind, avg=avg: ops.curve_score(s, kind, avg)[:2])
    for dt in (torch.float32, torch.float64):
        for k in (1, 3):
            st = [torch.rand(k, generator=g, dtype=torch.float64).to(dev, dt) + 1 for _ in range(5)]
            for kind in range(4):
                need = {0: 4, 1: 3}.get(kind, 5)
                for n in (torch.tensor([37.0], dtype=dt, device=dev), torch.tensor(37, device=dev), 37):
                    for mo in range(3):
                        def reg(st=st[:need], kind=kind, n=n, mo=mo, k=k):
                            out = ops.regression_compute(kind, st, n, mo, 0.3)
                            # out[k] (the average) is left unset for raw_values
                            return (out[:k], out[k + 1 :]) if mo == 0 else out

                        calls.append(reg)
    for dt in (torch.float32, torch.float64):
        for k in (1, 5):
            a = (torch.rand(k, generator=g, dtype=torch.float64) * 100).to(dev, dt)
            for b in (torch.tensor(37, device=dev), torch.tensor(3.5, dtype=dt, device=dev),
                      (torch.rand(k, generator=g, dtype=torch.float64) + 0.5).to(dev, dt)):
                for sq in (False, True):
                    calls.append(lambda a=a.squeeze() if k == 1 else a, b=b.squeeze() if k == 1 else b, sq=sq:
                                 ops.ratio(a, b, sq))
    for c in (1, 7, 300):
        # macro = mean of fp32-cast counts: bit-identical to ATen while the sums stay below 2^24 (beyond that the
        # task kernel sums exactly in int64 and rounds once, ATen rounds per partial sum)
        st = [torch.randint(0, 2**24 // 600, (c,), generator=g).to(dev) for _ in range(4)]
        for avg in ("micro", "macro", "none"):
            calls.append(lambda st=st, avg=avg: ops.stat_scores_output(*st, avg) if ops._RECORDER is not None else
                         _stat_scores_ref(*st, avg))
    eager = [c() for c in calls]
    with ops.fused_compute(poison=True) as rec:
        fused = [c() for c in calls]
    assert rec.flush() == len(calls)
    torch.cuda.synchronize()

    def same(a, b):
        if isinstance(a, (list, tuple)):
            return all(same(x, y) for x, y in zip(a, b))
        return torch.allclose(a, b, rtol=0, atol=0, equal_nan=True)

    bad = [i for i, (a, b) in enumerate(zip(eager, fused)) if not same(a, b)]
    assert not bad, bad


def test_graphed_compute_fuses_the_reductions():
    from torchmetrics_amd.utils.graphs import GraphedCompute

    cls, reg = _collection("cuda")
    lg, lb, x, y = _batch(7)
    cls.update(lg, lb)
    reg.update(x, y)
    g_cls, g_reg = GraphedCompute(cls), GraphedCompute(reg)
    assert g_cls._fusable >= {"acc", "prec", "f1", "spec", "jacc", "mcc", "kappa", "auroc", "ap"}
    assert g_reg._fusable >= {"r2", "pearson", "ev", "mse", "mae"}
    assert g_cls._fusable >= {"stat"}
