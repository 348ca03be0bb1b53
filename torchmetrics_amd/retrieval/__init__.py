"""Retrieval module metrics (parity: reference ``S/retrieval/__init__.py``)."""
from torchmetrics_amd.retrieval.base import RetrievalMetric
from torchmetrics_amd.retrieval.metrics import (
    RetrievalAUROC,
    RetrievalFallOut,
    RetrievalHitRate,
    RetrievalMAP,
    RetrievalMRR,
    RetrievalNormalizedDCG,
    RetrievalPrecision,
    RetrievalPrecisionRecallCurve,
    RetrievalRecall,
    RetrievalRecallAtFixedPrecision,
    RetrievalRPrecision,
)

__all__ = [k for k in dir() if k.startswith("Retrieval")]
