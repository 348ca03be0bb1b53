"""Text metrics (reference ``S/text/__init__.py``)."""
from torchmetrics_amd.text.scores import *  # noqa: F401,F403
from torchmetrics_amd.text.scores import __all__  # noqa: F401
