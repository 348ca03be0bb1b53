"""Native ``forward`` (``csrc/bindings/fastcall.cpp`` ``NativeForward`` + ``csrc/classification/forward.hip``).

Every batch value and the accumulated state equal the Python ``Metric.forward`` path (which follows the reference's
``_forward_reduce_state_update``, S/metric.py:353-391) and an fp64 CPU computation, for the confusion matrix and the
stat-score family (multiclass micro / macro / weighted / none, binary, multilabel; bf16 / fp16 / fp32 preds, int64 /
int32 targets, ignore_index).  Calls off the fast path (dist_sync_on_step, compute_on_cpu, held states, autograd-free
fallbacks, overridden update) give the reference result through ``Metric.forward``.
"""
import pickle

import pytest
import torch

import torchmetrics_amd as tm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pair(m_gpu, m_cpu, batches, dtype=torch.float32):
    vals = []
    for p, t in batches:
        a = m_gpu(p.to(DEV, dtype), t.to(DEV))
        b = m_cpu(p.to(dtype), t)
        vals.append((a, b))
    return vals


def _check(m_gpu, m_cpu, vals, atol=1e-6):
    for a, b in vals:
        assert a.shape == b.shape, (a.shape, b.shape)
        torch.testing.assert_close(a.cpu().to(b.dtype), b, atol=atol, rtol=1e-5)
    torch.testing.assert_close(m_gpu.compute().cpu(), m_cpu.compute(), atol=atol, rtol=1e-5)


def _mc_batches(C, n=4, rows=513, seed=0, ignore=None):
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(n):
        p = torch.randn(rows + i, C, generator=g)
        t = torch.randint(0, C, (rows + i,), generator=g)
        if ignore is not None:
            t[::7] = ignore
        out.append((p, t))
    return out


STAT_CLASSES = [tm.classification.MulticlassAccuracy, tm.classification.MulticlassPrecision,
                tm.classification.MulticlassRecall, tm.classification.MulticlassF1Score,
                tm.classification.MulticlassSpecificity, tm.classification.MulticlassHammingDistance]


@pytest.mark.parametrize("cls", STAT_CLASSES)
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", None])
@pytest.mark.parametrize("C", [10, 1000])
def test_multiclass_stat_forward(cls, average, C):
    m = cls(C, average=average).to(DEV)
    assert type(m.forward).__name__ == "NativeForward"
    ref = cls(C, average=average)
    vals = _pair(m, ref, _mc_batches(C), torch.bfloat16)
    assert m.forward.native_calls == 3, m.forward.decline_line  # the first call builds the workspace / validation word in Python
    _check(m, ref, vals)


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32])
def test_fbeta_forward_dtypes_and_ignore(dtype, tdtype):
    C = 37
    m = tm.classification.MulticlassFBetaScore(2.0, C, ignore_index=3).to(DEV)
    ref = tm.classification.MulticlassFBetaScore(2.0, C, ignore_index=3)
    batches = [(p, t.to(tdtype)) for p, t in _mc_batches(C, ignore=3)]
    vals = _pair(m, ref, batches, dtype)
    assert m.forward.native_calls == 3, m.forward.decline_line
    _check(m, ref, vals)


@pytest.mark.parametrize("cls", [tm.classification.BinaryAccuracy, tm.classification.BinaryF1Score,
                                 tm.classification.BinarySpecificity, tm.classification.BinaryHammingDistance])
@pytest.mark.parametrize("logits", [False, True])
def test_binary_stat_forward(cls, logits):
    g = torch.Generator().manual_seed(1)
    batches = []
    for i in range(4):
        p = torch.randn(1000 + i, generator=g) if logits else torch.rand(1000 + i, generator=g)
        batches.append((p, torch.randint(0, 2, (1000 + i,), generator=g)))
    m, ref = cls().to(DEV), cls()
    assert type(m.forward).__name__ == "NativeForward"
    vals = _pair(m, ref, batches)
    assert m.forward.native_calls == 3, m.forward.decline_line
    _check(m, ref, vals)


@pytest.mark.parametrize("cls", [tm.classification.MultilabelAccuracy, tm.classification.MultilabelF1Score,
                                 tm.classification.MultilabelPrecision])
@pytest.mark.parametrize("average", ["micro", "macro", "weighted", None])
def test_multilabel_stat_forward(cls, average):
    L = 19
    g = torch.Generator().manual_seed(2)
    batches = [(torch.rand(300 + i, L, generator=g), torch.randint(0, 2, (300 + i, L), generator=g)) for i in range(4)]
    m, ref = cls(L, average=average).to(DEV), cls(L, average=average)
    vals = _pair(m, ref, batches, torch.bfloat16)
    assert m.forward.native_calls == 3, m.forward.decline_line
    _check(m, ref, vals)


@pytest.mark.parametrize("C", [5, 1000])
@pytest.mark.parametrize("ignore_index", [None, 2])
def test_confmat_forward(C, ignore_index):
    m = tm.MulticlassConfusionMatrix(C, ignore_index=ignore_index).to(DEV)
    assert type(m.forward).__name__ == "NativeForward"
    ref = tm.MulticlassConfusionMatrix(C, ignore_index=ignore_index)
    batches = _mc_batches(C, ignore=ignore_index)
    vals = _pair(m, ref, batches, torch.bfloat16)
    assert m.forward.native_calls == 3, m.forward.decline_line
    _check(m, ref, vals, atol=0)
    # against a direct fp32 bincount of the whole stream
    p = torch.cat([b[0] for b in batches]).to(torch.bfloat16).float()
    t = torch.cat([b[1] for b in batches])
    keep = t != ignore_index if ignore_index is not None else torch.ones_like(t, dtype=torch.bool)
    direct = torch.bincount(t[keep] * C + p.argmax(1)[keep], minlength=C * C).reshape(C, C)
    assert torch.equal(m.compute().cpu(), direct)


def test_held_states_fall_back_and_stay_unchanged():
    """The reference merges out of place: a held compute() result (the confusion matrix IS the state) or a held view
    must not change under forward -- the native path declines and Metric.forward merges out of place."""
    C = 8
    batches = _mc_batches(C, n=3)
    m = tm.MulticlassConfusionMatrix(C).to(DEV)
    m(batches[0][0].to(DEV), batches[0][1].to(DEV))
    held = m.compute()
    before = held.clone()
    m(batches[1][0].to(DEV), batches[1][1].to(DEV))
    assert torch.equal(held, before)
    a = tm.MulticlassAccuracy(C, average=None).to(DEV)
    a(batches[0][0].to(DEV), batches[0][1].to(DEV))
    view = a.tp[2:]
    vb = view.clone()
    calls = a.forward.native_calls
    a(batches[1][0].to(DEV), batches[1][1].to(DEV))
    assert torch.equal(view, vb) and a.forward.native_calls == calls
    del view
    a(batches[2][0].to(DEV), batches[2][1].to(DEV))
    assert a.forward.native_calls == calls + 1  # nothing held any more: native again


@pytest.mark.parametrize("kwargs", [{"dist_sync_on_step": True}, {"compute_on_cpu": True}])
def test_forward_preconditions_fall_back(kwargs):
    C = 10
    m = tm.MulticlassAccuracy(C, **kwargs).to(DEV)
    ref = tm.MulticlassAccuracy(C)
    vals = _pair(m, ref, _mc_batches(C))
    assert m.forward.native_calls == 0
    _check(m, ref, vals)


def test_forward_autograd_inputs_and_samplewise():
    C = 10
    p, t = _mc_batches(C, n=1)[0]
    m = tm.MulticlassAccuracy(C).to(DEV)
    x = p.to(DEV).requires_grad_(True)
    m(x, t.to(DEV))
    v = m(x, t.to(DEV))
    torch.testing.assert_close(v.cpu(), tm.functional.multiclass_accuracy(p, t, C))
    s = tm.MulticlassAccuracy(C, multidim_average="samplewise").to(DEV)
    assert "forward" not in s.__dict__  # samplewise: Metric.forward


def test_forward_errors_surface_at_compute():
    C = 10
    m = tm.MulticlassAccuracy(C).to(DEV)
    p, t = _mc_batches(C, n=1)[0]
    m(p.to(DEV), t.to(DEV))
    bad = t.clone()
    bad[3] = C + 4
    m(p.to(DEV), bad.to(DEV))
    assert m.forward.native_calls == 1
    with pytest.raises(RuntimeError, match="more unique values in `target`"):
        m.compute()


class _Shifted(tm.MulticlassAccuracy):
    def update(self, preds, target):
        super().update(preds, (target + 1) % self.num_classes)


def test_overrides_and_pickle():
    assert "forward" not in _Shifted(5).to(DEV).__dict__
    m = tm.MulticlassF1Score(7).to(DEV)
    p, t = _mc_batches(7, n=2)[0]
    m(p.to(DEV), t.to(DEV))
    for other in (pickle.loads(pickle.dumps(m)), m.clone()):
        assert type(other.forward).__name__ == "NativeForward"
        other(p.to(DEV), t.to(DEV))
        other(p.to(DEV), t.to(DEV))
        assert other.forward.native_calls >= 1
        torch.testing.assert_close(other.compute().cpu(), tm.functional.multiclass_f1_score(
            torch.cat([p] * 3), torch.cat([t] * 3), 7))


def test_collection_forward_uses_native_members():
    C = 10
    coll = tm.MetricCollection({"acc": tm.MulticlassAccuracy(C), "cm": tm.MulticlassConfusionMatrix(C)}).to(DEV)
    ref = tm.MetricCollection({"acc": tm.MulticlassAccuracy(C), "cm": tm.MulticlassConfusionMatrix(C)})
    for p, t in _mc_batches(C):
        a = coll(p.to(DEV), t.to(DEV))
        b = ref(p, t)
        for k in b:
            torch.testing.assert_close(a[k].cpu(), b[k])
    out, exp = coll.compute(), ref.compute()
    for k in exp:
        torch.testing.assert_close(out[k].cpu(), exp[k])


@pytest.mark.parametrize("make", [
    lambda: tm.classification.MulticlassAccuracy(10, average="micro"),
    lambda: tm.classification.MulticlassF1Score(1000, ignore_index=3),
    lambda: tm.classification.MulticlassStatScores(37, average=None),
    lambda: tm.classification.BinaryPrecision(),
    lambda: tm.classification.MultilabelRecall(19),
])
def test_native_stat_update(make):
    m, ref = make().to(DEV), make()
    assert type(m.update).__name__ == "NativeUpdate"
    g = torch.Generator().manual_seed(11)
    for i in range(4):
        if isinstance(ref, tm.classification.MulticlassStatScores):
            C = ref.num_classes
            p, t = torch.randn(300 + i, C, generator=g).to(torch.bfloat16), torch.randint(0, C, (300 + i,), generator=g)
        elif isinstance(ref, tm.classification.MultilabelStatScores):
            p, t = torch.rand(300 + i, 19, generator=g), torch.randint(0, 2, (300 + i, 19), generator=g)
        else:
            p, t = torch.randn(300 + i, generator=g), torch.randint(0, 2, (300 + i,), generator=g)
        m.update(p.to(DEV), t.to(DEV))
        ref.update(p, t)
    assert m.update.native_calls == 3 and m.update_count == 4
    torch.testing.assert_close(m.compute().cpu(), ref.compute())


def test_native_stat_update_fallbacks():
    m = tm.classification.MulticlassAccuracy(10, top_k=2).to(DEV)
    p, t = torch.randn(64, 10), torch.randint(0, 10, (64,))
    m.update(p.to(DEV), t.to(DEV))
    m.update(p.to(DEV), t.to(DEV))
    assert m.update.native_calls == 0  # top_k > 1: the Python update (fused top-k kernel)
    torch.testing.assert_close(m.compute().cpu(), tm.functional.multiclass_accuracy(p, t, 10, top_k=2))
    assert type(_Shifted(5).to(DEV).update).__name__ != "NativeUpdate"
