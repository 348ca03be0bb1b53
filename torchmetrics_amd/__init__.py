"""torchmetrics_amd: an MI355X-native (ROCm / CDNA4) metrics framework with the torchmetrics 1.4 API.

Root namespace mirrors reference ``S/__init__.py:23-151``.
"""
import logging as __logging

from torchmetrics_amd.__about__ import __version__  # noqa: F401

_logger = __logging.getLogger("torchmetrics_amd")
_logger.addHandler(__logging.StreamHandler())
_logger.setLevel(__logging.INFO)

from torchmetrics_amd import _module_aliases  # noqa: E402

_module_aliases.install()

from torchmetrics_amd import functional  # noqa: E402,F401
from torchmetrics_amd.aggregation import (  # noqa: E402
    CatMetric,
    MaxMetric,
    MeanMetric,
    MinMetric,
    RunningMean,
    RunningSum,
    SumMetric,
)
from torchmetrics_amd.classification import *  # noqa: E402,F401,F403
from torchmetrics_amd.collections import MetricCollection  # noqa: E402
from torchmetrics_amd.metric import CompositionalMetric, Metric  # noqa: E402
from torchmetrics_amd.regression import *  # noqa: E402,F401,F403
from torchmetrics_amd.wrappers import (  # noqa: E402
    BootStrapper,
    ClasswiseWrapper,
    MetricTracker,
    MinMaxMetric,
    MultioutputWrapper,
    MultitaskWrapper,
)
from torchmetrics_amd.nominal import (  # noqa: E402
    CramersV,
    FleissKappa,
    PearsonsContingencyCoefficient,
    TheilsU,
    TschuprowsT,
)
from torchmetrics_amd._deprecated import ROOT_CLASSES as __ROOT_CLASSES  # noqa: E402
from torchmetrics_amd._deprecated import deprecated_class as __deprecated_class  # noqa: E402

# deprecated root aliases (audio / detection / image / retrieval / text), reference ``S/__init__.py:33-151``
for __name, __domain in __ROOT_CLASSES.items():
    globals()[__name] = __deprecated_class(__name, __domain)
del __name, __domain
