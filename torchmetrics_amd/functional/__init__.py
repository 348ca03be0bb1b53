"""Functional (stateless) metrics (parity: reference ``F/__init__.py``)."""
from torchmetrics_amd.functional.classification import *  # noqa: F401,F403
from torchmetrics_amd.functional.regression import *  # noqa: F401,F403
from torchmetrics_amd.functional.retrieval import *  # noqa: F401,F403
from torchmetrics_amd.functional.image import *  # noqa: F401,F403
from torchmetrics_amd.functional.detection import *  # noqa: F401,F403
from torchmetrics_amd.functional.clustering import *  # noqa: F401,F403
from torchmetrics_amd.functional.nominal import *  # noqa: F401,F403
from torchmetrics_amd.functional.pairwise import *  # noqa: F401,F403
from torchmetrics_amd.functional.text import *  # noqa: F401,F403
from torchmetrics_amd.functional.audio import *  # noqa: F401,F403
from torchmetrics_amd.functional.multimodal import *  # noqa: F401,F403

from torchmetrics_amd._deprecated import FUNCTIONAL_ROOT as _FUNCTIONAL_ROOT  # noqa: E402
from torchmetrics_amd._deprecated import deprecated_function as _deprecated_function  # noqa: E402

# deprecated root aliases of domain functionals, reference ``F/__init__.py`` (``F/*/_deprecated.py``)
for _name, _domain in _FUNCTIONAL_ROOT.items():
    try:
        globals()[_name] = _deprecated_function(_name, _domain)
    except AttributeError:  # optional backend (e.g. transformers) not importable
        pass
