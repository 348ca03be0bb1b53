"""Native ``update`` entry point (``csrc/bindings/fastcall.cpp`` ``NativeUpdate``) for MulticlassConfusionMatrix.

CPU part: the callable is bound to the metric's ``__dict__`` and hands every input off its fast path (CPU tensors,
kwargs) to the Python ``update``; it unwraps like the Python wrapper (``inspect.signature`` / ``is_overridden``) and
survives pickling / cloning.  GPU part: the fast path itself -- results equal to the Python path for every input
dtype, ``ignore_index`` / ``validate_args=False``, deferred validation errors, ``forward``, device moves.
"""
import inspect
import pickle

import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.checks import is_overridden


def _force_native(m):
    assert ops.load_native(strict=False)
    fast = ops._fast_mod.confmat_updater(m.__dict__, m.__dict__["update"])
    m.__dict__["update"] = fast
    return fast


def test_cpu_inputs_take_the_python_path():
    m = tm.MulticlassConfusionMatrix(5)
    fast = _force_native(m)
    g = torch.Generator().manual_seed(0)
    p, t = torch.randn(30, 5, generator=g), torch.randint(0, 5, (30,), generator=g)
    m.update(p[:10], t[:10])
    m.update(preds=p[10:], target=t[10:])
    assert m.update_count == 2 and fast.native_calls == 0
    torch.testing.assert_close(m.compute(), tm.functional.multiclass_confusion_matrix(p, t, 5))
    assert str(inspect.signature(m.update)) == "(preds: torch.Tensor, target: torch.Tensor) -> None"
    assert is_overridden("update", m, Metric)
    with pytest.raises(ValueError, match="number of classes"):
        m.update(torch.randn(4, 6), torch.randint(0, 5, (4,)))


def test_pickle_and_clone_reinstall_hook():
    m = tm.MulticlassConfusionMatrix(4)
    m.update(torch.randn(8, 4), torch.randint(0, 4, (8,)))
    for other in (pickle.loads(pickle.dumps(m)), m.clone()):
        other.update(torch.randn(8, 4), torch.randint(0, 4, (8,)))
        assert int(other.compute().sum()) == 16


@pytest.mark.gpu
@pytest.mark.parametrize("pdtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("tdtype", [torch.int64, torch.int32])
@pytest.mark.parametrize("ignore_index", [None, 3])
def test_gpu_fast_path_matches_python_path(pdtype, tdtype, ignore_index):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    C = 37
    native = tm.MulticlassConfusionMatrix(C, ignore_index=ignore_index).to(dev)
    assert type(native.update).__name__ == "NativeUpdate"
    ref = tm.MulticlassConfusionMatrix(C, ignore_index=ignore_index)
    for i in range(4):
        p = torch.randn(257 + i, C, generator=g).to(pdtype)
        t = torch.randint(0, C, (257 + i,), generator=g).to(tdtype)
        native.update(p.to(dev), t.to(dev))
        ref.update(p, t)
    assert native.update.native_calls == 3  # the first call creates the validation word in Python
    assert native.update_count == 4
    assert torch.equal(native.compute().cpu(), ref.compute())


@pytest.mark.gpu
def test_gpu_fast_path_semantics():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(8)
    m = tm.MulticlassConfusionMatrix(10).to(dev)
    p, t = torch.randn(64, 10, generator=g).to(dev), torch.randint(0, 10, (64,), generator=g).to(dev)
    m.update(p, t)
    m.update(p, t)
    assert m.update.native_calls == 1
    c1 = m.compute().clone()  # compute() returns the state itself (as the reference)
    m.update(p, t)
    assert m._computed is None  # bookkeeping done natively
    assert int(m.compute().sum()) == 192 and int(c1.sum()) == 128
    # deferred validation: an out-of-range target raises at compute with the reference's message
    bad = t.clone()
    bad[5] = 12
    m.update(p, bad)
    with pytest.raises(RuntimeError, match="more unique values in `target`"):
        m.compute()
    # shape errors fall through to the Python validation (reference ValueError)
    with pytest.raises(ValueError):
        m.update(p[:, :9], t)
    # forward() and validate_args=False go through the same entry
    m2 = tm.MulticlassConfusionMatrix(10, validate_args=False).to(dev)
    batch = m2(p, t)
    assert int(batch.sum()) == 64 and int(m2.compute().sum()) == 64
    m2.update(p, t)
    assert m2.update.native_calls >= 1
    # moving the metric keeps the path consistent (state on CPU -> Python path)
    m3 = tm.MulticlassConfusionMatrix(10).to(dev)
    m3.update(p, t)
    m3 = m3.to("cpu")
    m3.update(p.cpu(), t.cpu())
    assert int(m3.compute().sum()) == 128


def test_reset_refills_unobserved_state_in_place():
    """``Metric.reset`` refills a state's own memory only when nothing can observe it (no other reference, no view);
    otherwise it allocates a fresh default like the reference (S/metric.py:673-688)."""
    g = torch.Generator().manual_seed(1)
    m = tm.MulticlassConfusionMatrix(5)
    m.update(torch.randn(10, 5, generator=g), torch.randint(0, 5, (10,), generator=g))
    ident = id(m.confmat)
    m.reset()
    assert id(m.confmat) == ident and int(m.confmat.sum()) == 0
    m.update(torch.randn(10, 5, generator=g), torch.randint(0, 5, (10,), generator=g))
    held = m.compute()
    m.reset()
    assert int(held.sum()) == 10 and int(m.confmat.sum()) == 0  # a returned result is never clobbered
    m.update(torch.randn(10, 5, generator=g), torch.randint(0, 5, (10,), generator=g))
    view = m.confmat[0]
    before = view.clone()
    m.reset()
    assert torch.equal(view, before)  # nor is a view of the old state
    mx = tm.MaxMetric()
    mx.update(torch.tensor(3.0))
    mx.reset()
    assert float(mx.max_value) == float("-inf")  # non-zero defaults are restored too


class _ShiftedConfmat(tm.MulticlassConfusionMatrix):
    """A user subclass that preprocesses in its own update (the reference always runs it)."""

    def update(self, preds, target):
        super().update(preds, (target + 1) % self.num_classes)


def test_subclass_update_is_not_bypassed_cpu():
    m = _ShiftedConfmat(4)
    assert "update" not in m.__dict__ or type(m.__dict__["update"]).__name__ != "NativeUpdate"
    p, t = torch.randn(16, 4), torch.randint(0, 4, (16,))
    m.update(p, t)
    torch.testing.assert_close(m.compute(), tm.functional.multiclass_confusion_matrix(p, (t + 1) % 4, 4))
    other = pickle.loads(pickle.dumps(m))
    assert type(other.__dict__.get("update")).__name__ != "NativeUpdate"


@pytest.mark.gpu
def test_subclass_update_is_not_bypassed_gpu():
    dev = torch.device("cuda", 0)
    m = _ShiftedConfmat(6).to(dev)
    assert type(m.update).__name__ != "NativeUpdate"
    g = torch.Generator().manual_seed(3)
    p, t = torch.randn(100, 6, generator=g), torch.randint(0, 6, (100,), generator=g)
    m.update(p.to(dev), t.to(dev))
    ref = tm.functional.multiclass_confusion_matrix(p, (t + 1) % 6, 6)
    assert torch.equal(m.compute().cpu(), ref)
    assert type(tm.MulticlassConfusionMatrix(6).to(dev).update).__name__ == "NativeUpdate"


@pytest.mark.gpu
def test_native_update_stays_on_with_roctx_ranges():
    """Profiler ranges are opened by the native entry point itself (csrc/bindings/fastcall.cpp RangeScope): turning
    them on keeps the production fast path (verdict r4: ranges used to switch the native update off)."""
    from torchmetrics_amd.utils import profiling

    profiling.enable(True)
    try:
        m = tm.MulticlassConfusionMatrix(num_classes=7).to("cuda")
        assert type(m.update).__name__ == "NativeUpdate"
        assert m.update.range_name == "tm.update/MulticlassConfusionMatrix"
        p, t = torch.randn(64, 7, device="cuda"), torch.randint(0, 7, (64,), device="cuda")
        for _ in range(3):
            m.update(p, t)
        assert m.update.native_calls > 0
        f = tm.MulticlassAccuracy(num_classes=7).to("cuda")
        f(p, t)
        f(p, t)
        assert type(f.forward).__name__ == "NativeForward" and f.forward.range_name == "tm.forward/MulticlassAccuracy"
        assert f.forward.native_calls > 0
    finally:
        profiling.enable(False)


@pytest.mark.gpu
def test_read_word_matches_item_and_leaves_stream_idle():
    """ops.read_word (mapped host memory + stream sync) returns the word's value and raises nothing on a clean word;
    compute() still raises a deferred target-range error through it."""
    w = torch.tensor([0x25], dtype=torch.int32, device="cuda")
    assert ops.read_word(w) == 0x25
    w.zero_()
    assert ops.read_word(w) == 0
    m = tm.MulticlassConfusionMatrix(num_classes=5).to("cuda")
    p = torch.randn(16, 5, device="cuda")
    m.update(p, torch.randint(0, 5, (16,), device="cuda"))
    m.update(p, torch.full((16,), 7, device="cuda"))  # out of range: the kernel flags it
    with pytest.raises(RuntimeError):
        m.compute()
