"""Text metrics (reference ``S/text/__init__.py``)."""
from torchmetrics_amd.text.scores import *  # noqa: F401,F403
from torchmetrics_amd.text.scores import __all__ as _base_all
from torchmetrics_amd.utilities.imports import _TRANSFORMERS_AVAILABLE

__all__ = list(_base_all)
if _TRANSFORMERS_AVAILABLE:
    from torchmetrics_amd.text.model_based import BERTScore, InfoLM  # noqa: F401

    __all__ += ["BERTScore", "InfoLM"]
