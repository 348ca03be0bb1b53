"""The native forward's aliasing test (``csrc/bindings/fastcall.cpp`` ``states_unobserved``), probed on CPU tensors.

The native ``forward`` merges the batch into the global states in place, so it may only run when nothing outside the
metric can observe them (the reference merges out of place, S/metric.py:329-352).  torch 2.10 keeps the Python
wrapper of a storage alive (and holding one reference) once ``untyped_storage()`` has been called, and keeps a view
base's Python wrapper alive for its views: the probe must count both as the metric's own, and still see a held
view, a held ``compute()`` result or a held arena buffer.
"""
import pytest
import torch

import torchmetrics_amd as tm
from torchmetrics_amd import ops

pytestmark = pytest.mark.skipif(not ops.native_available(), reason="native library not built")


def _probe(state, keys):
    return ops._fast()._states_unobserved(state, tuple(keys))


def test_plain_state_storage_wrapper_and_views():
    x = torch.zeros(3)
    d = {"_defaults": {"x": None}, "x": x}
    del x
    assert _probe(d, ["x"])[0]
    s = d["x"].untyped_storage()  # the preserved storage wrapper is not an outside observer
    assert _probe(d, ["x"])[0]
    del s
    v = d["x"][1:]
    assert _probe(d, ["x"]) == (False, 3, 2)  # a view keeps the state's own Python object referenced
    del v
    assert _probe(d, ["x"])[0]
    held = d["x"]
    assert not _probe(d, ["x"])[0]
    del held


def test_confmat_after_forward_and_held_compute():
    m = tm.MulticlassConfusionMatrix(5)
    m(torch.randn(10, 5), torch.randint(0, 5, (10,)))
    assert _probe(m.__dict__, ["confmat"])[0]
    h = m.compute()  # the confusion matrix IS the state
    assert not _probe(m.__dict__, ["confmat"])[0]
    del h


def test_packed_arena_states():
    a = tm.classification.MulticlassAccuracy(10)
    a(torch.randn(10, 10), torch.randint(0, 10, (10,)))
    keys = ["tp", "fp", "tn", "fn"]
    assert a.tp._base is not None  # the four states are views of one arena buffer
    assert _probe(a.__dict__, keys)[0]
    v = a.fn[3:]
    ok, why, _ = _probe(a.__dict__, keys)
    assert not ok and why == 6
    del v
    assert _probe(a.__dict__, keys)[0]
    b = a.tp._base
    assert _probe(a.__dict__, keys)[:2] == (False, 7)
    del b
    assert _probe(a.__dict__, keys)[0]


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["attribute", "metric_state", "compute", "state_dict_keep_vars", "arena_view"])
def test_held_state_never_changes_under_native_forward(how):
    """The reference's reduce-state forward (``S/metric.py:329-352``) re-binds fresh state tensors, so a state object
    the user holds keeps its value.  The ROCm native forward merges in place only when nothing outside holds a state;
    whichever way a state was handed out -- an attribute read, ``metric_state``, a ``compute()`` result that IS the
    state, ``state_dict(keep_vars=True)`` or a view -- the held object must not change, and the metric's own states
    and batch values must equal a CPU run."""
    dev = "cuda"
    g = torch.Generator().manual_seed(2)
    batches = [(torch.randn(257, 6, generator=g), torch.randint(0, 6, (257,), generator=g)) for _ in range(4)]
    for make in (lambda: tm.MulticlassConfusionMatrix(6), lambda: tm.classification.MulticlassAccuracy(6)):
        m, ref = make().to(dev), make()
        m.persistent(True)
        for i, (p, t) in enumerate(batches):
            attr = "confmat" if hasattr(m, "confmat") else "tp"
            if how == "attribute":
                held = getattr(m, attr)
            elif how == "metric_state":
                held = m.metric_state[attr]
            elif how == "compute":
                held = m.compute() if i else getattr(m, attr)
            elif how == "state_dict_keep_vars":
                held = m.state_dict(keep_vars=True)[attr]
            else:
                held = getattr(m, attr)[1:]
            snap = held.clone()
            out = m(p.to(dev), t.to(dev))
            ref_out = ref(p, t)
            assert torch.equal(held, snap), f"{how}: a held state changed under forward (batch {i})"
            torch.testing.assert_close(out.cpu(), ref_out)
            del held
        torch.testing.assert_close(m.compute().cpu(), ref.compute())
