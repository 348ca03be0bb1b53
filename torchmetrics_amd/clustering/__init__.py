"""Clustering metrics (reference ``S/clustering/__init__.py``)."""
from torchmetrics_amd.clustering.scores import *  # noqa: F401,F403
from torchmetrics_amd.clustering.scores import __all__  # noqa: F401
