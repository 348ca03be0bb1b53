"""Regression module metrics (parity: reference ``S/regression/__init__.py``)."""
from torchmetrics_amd.regression.correlation import (
    ConcordanceCorrCoef,
    CosineSimilarity,
    KendallRankCorrCoef,
    KLDivergence,
    PearsonCorrCoef,
    SpearmanCorrCoef,
)
from torchmetrics_amd.regression.streaming import (
    CriticalSuccessIndex,
    ExplainedVariance,
    LogCoshError,
    MeanAbsoluteError,
    MeanAbsolutePercentageError,
    MeanSquaredError,
    MeanSquaredLogError,
    MinkowskiDistance,
    R2Score,
    RelativeSquaredError,
    SymmetricMeanAbsolutePercentageError,
    TweedieDevianceScore,
    WeightedMeanAbsolutePercentageError,
)

__all__ = [k for k in dir() if k[0].isupper()]
