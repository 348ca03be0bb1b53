"""Metric wrappers (parity: reference ``S/wrappers/__init__.py``)."""
from torchmetrics_amd.wrappers.abstract import WrapperMetric
from torchmetrics_amd.wrappers.bootstrapping import BootStrapper
from torchmetrics_amd.wrappers.classwise import ClasswiseWrapper
from torchmetrics_amd.wrappers.feature_share import FeatureShare
from torchmetrics_amd.wrappers.minmax import MinMaxMetric
from torchmetrics_amd.wrappers.multioutput import MultioutputWrapper
from torchmetrics_amd.wrappers.multitask import MultitaskWrapper
from torchmetrics_amd.wrappers.running import Running
from torchmetrics_amd.wrappers.tracker import MetricTracker

__all__ = [
    "BootStrapper",
    "ClasswiseWrapper",
    "FeatureShare",
    "MetricTracker",
    "MinMaxMetric",
    "MultioutputWrapper",
    "MultitaskWrapper",
    "Running",
    "WrapperMetric",
]
