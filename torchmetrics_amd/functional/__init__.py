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
