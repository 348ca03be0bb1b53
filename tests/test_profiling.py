"""roctx lifecycle ranges (``torchmetrics_amd/utils/profiling.py``): off by default; when on, update / forward /
compute / collection compute / sync open and close balanced ranges with the documented names (recorded here through a
stand-in for the roctx library), and torch.profiler sees them as record_function ranges."""
import torch

import torchmetrics_amd as tm
from torchmetrics_amd.utils import profiling
from tests.helpers import run_ddp


def _capture(monkeypatch):
    events = []
    monkeypatch.setattr(profiling, "_push", lambda name: events.append(("push", name)))
    monkeypatch.setattr(profiling, "_pop", lambda: events.append(("pop", None)))
    monkeypatch.setattr(profiling, "ENABLED", True)
    return events


def _balanced(events):
    depth = 0
    for kind, _ in events:
        depth += 1 if kind == "push" else -1
        assert depth >= 0
    return depth == 0


def test_off_by_default_and_real_binding(monkeypatch):
    import os

    assert profiling.ENABLED == (os.environ.get("TORCHMETRICS_AMD_ROCTX", "0") not in ("0", "", "false", "False"))
    monkeypatch.setattr(profiling, "_push", None)
    monkeypatch.setattr(profiling, "_pop", None)
    monkeypatch.setattr(profiling, "ENABLED", False)
    profiling.enable(True)  # binds the rocprofiler-sdk roctx library (or torch's roctx) and pushes / pops for real
    with profiling.range("tm.test"):
        pass
    profiling.enable(False)
    assert profiling._push is not None


def test_metric_lifecycle_ranges(monkeypatch):
    events = _capture(monkeypatch)
    m = tm.MulticlassAccuracy(5)
    p, t = torch.randn(8, 5), torch.randint(0, 5, (8,))
    m.update(p, t)
    m(p, t)
    m.compute()
    coll = tm.MetricCollection([tm.MulticlassAccuracy(5), tm.MulticlassF1Score(5)])
    coll.update(p, t)
    coll.compute()
    names = [n for k, n in events if k == "push"]
    assert "tm.update/MulticlassAccuracy" in names and "tm.forward/MulticlassAccuracy" in names
    assert "tm.compute/MulticlassAccuracy" in names and "tm.collection.compute" in names
    assert _balanced(events)


def _sync_ranges(rank, world):
    events = []
    profiling._push = lambda name: events.append(("push", name))
    profiling._pop = lambda: events.append(("pop", None))
    profiling.ENABLED = True
    m = tm.MulticlassAccuracy(5)
    m.update(torch.randn(8, 5), torch.randint(0, 5, (8,)))
    m.compute()
    names = [n for k, n in events if k == "push"]
    assert any(n.startswith("tm.sync/") for n in names), names
    assert any(n.startswith("tm.sync.bucket/sum/int64/") for n in names), names
    assert _balanced(events)


def test_sync_bucket_ranges_two_ranks():
    run_ddp(_sync_ranges, world=2)


def test_torch_profiler_sees_ranges(monkeypatch):
    monkeypatch.setattr(profiling, "_push", lambda name: None)
    monkeypatch.setattr(profiling, "_pop", lambda: None)
    monkeypatch.setattr(profiling, "ENABLED", True)
    m = tm.MeanSquaredError()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        m.update(torch.randn(10), torch.randn(10))
        m.compute()
    keys = {e.key for e in prof.key_averages()}
    assert "tm.update/MeanSquaredError" in keys and "tm.compute/MeanSquaredError" in keys
