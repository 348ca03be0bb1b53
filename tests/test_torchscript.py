"""TorchScript contract: every public metric class scripts with ``torch.jit.script``, as the reference's tester checks
for each metric (``tests/unittests/helpers/testers.py:132-133``, ``bases/test_metric.py:359-361``).  The exceptions are
the classes the reference never scripts either: model-backed metrics (feature networks / HF models, its tests pass
``check_scriptable=False`` or use custom tests), ``CatMetric`` / ``RunningMean`` / ``RunningSum`` (not in its scripted
aggregation set), the wrappers its tests do not script, and the abstract bases.  On ROCm the native C++ ``update`` / ``forward`` entry points step aside
(``Metric.__prepare_scriptable__``)."""
import inspect

import pytest
import torch

import torchmetrics_amd as tm
from tests.test_class_attrs import METRIC_CLASSES, _ours

NOT_SCRIPTED = {
    # model-backed (feature extractors / pretrained networks; reference: custom tests or check_scriptable=False)
    "FrechetInceptionDistance", "KernelInceptionDistance", "InceptionScore",
    "MemorizationInformedFrechetInceptionDistance", "LearnedPerceptualImagePatchSimilarity", "PerceptualPathLength",
    "CLIPScore", "CLIPImageQualityAssessment", "BERTScore", "InfoLM", "PerceptualEvaluationSpeechQuality",
    # not in the reference's scripted set (tests/unittests/bases/test_aggregation.py:63-80)
    "CatMetric", "RunningMean", "RunningSum",
    # wrappers the reference never scripts (only MultioutputWrapper goes through its tester; MinMaxMetric passes
    # check_scriptable=False, tests/unittests/wrappers/test_minmax.py)
    "ClasswiseWrapper", "MinMaxMetric", "MultitaskWrapper", "Running", "BootStrapper",
    # abstract
    "Metric", "WrapperMetric",
}

_BY_NAME = {"beta": 2.0, "min_recall": 0.5, "min_precision": 0.5, "min_specificity": 0.5, "min_sensitivity": 0.5,
            "num_classes": 3, "num_labels": 3, "num_groups": 2, "num_outputs": 2, "task": "multiclass",
            "things": {0, 1}, "stuffs": {2}, "fs": 8000, "data_range": 1.0, "window": 3}


_SPECIAL = {
    "BaseAggregator": lambda: {"fn": "sum", "default_value": torch.tensor(0.0)},
    "MultioutputWrapper": lambda: {"base_metric": tm.MeanSquaredError(), "num_outputs": 2},
}


def _args(cls):
    if cls.__name__ in _SPECIAL:
        return _SPECIAL[cls.__name__]()
    fn = cls.__new__ if "__new__" in cls.__dict__ else cls.__init__
    kw = {}
    for p in list(inspect.signature(fn).parameters.values())[1:]:
        if p.kind in (p.VAR_KEYWORD, p.VAR_POSITIONAL) or p.default is not inspect.Parameter.empty:
            continue
        if p.name in ("base_metric", "metric"):
            kw[p.name] = tm.MulticlassAccuracy(3)
        elif p.name == "task_metrics":
            kw[p.name] = {"a": tm.MulticlassAccuracy(3)}
        else:
            kw[p.name] = _BY_NAME.get(p.name, 3)
    if "num_classes" in inspect.signature(fn).parameters and "task" in kw:
        kw["num_classes"] = 3
    return kw


CASES = [k for k in METRIC_CLASSES if k.split(":")[1] not in NOT_SCRIPTED]


@pytest.mark.parametrize("key", CASES, ids=[k.split(":")[1] + "@" + k.split(":")[0].split(".")[-1] for k in CASES])
def test_metric_class_scripts(key):
    cls = _ours(key)
    metric = cls(**_args(cls))
    scripted = torch.jit.script(metric)
    assert isinstance(scripted, torch.jit.ScriptModule)


class _ListMetric(tm.Metric):
    def __init__(self):
        super().__init__()
        self.add_state("x", [], dist_reduce_fx="cat")

    def update(self, v):
        self.x.append(v)

    def compute(self):
        return torch.cat(self.x).sum()


def test_list_state_metric_scripts():
    torch.jit.script(_ListMetric())


@pytest.mark.gpu
@pytest.mark.parametrize("make", [lambda: tm.MulticlassAccuracy(5), lambda: tm.MulticlassConfusionMatrix(5)])
def test_scripting_with_native_entry_points(make):
    m = make().cuda()
    p, t = torch.randn(16, 5, device="cuda"), torch.randint(0, 5, (16,), device="cuda")
    m(p, t)
    fwd, upd = type(m.forward).__name__, type(m.update).__name__
    calls = m.update.native_calls if upd == "NativeUpdate" else None
    torch.jit.script(m)
    # scripting works on a copy: the eager metric keeps its native entry points and they keep running
    assert type(m.forward).__name__ == fwd and type(m.update).__name__ == upd
    m(p, t)
    if calls is not None:
        m.update(p, t)
        assert m.update.native_calls > calls
        m2 = make().cuda()
        m2(p, t)
        m2(p, t)
        m2.update(p, t)
        m = m2
    ref = make()
    ref(p.cpu(), t.cpu())
    ref(p.cpu(), t.cpu())
    if calls is not None:
        ref.update(p.cpu(), t.cpu())
    torch.testing.assert_close(m.compute().cpu(), ref.compute())
