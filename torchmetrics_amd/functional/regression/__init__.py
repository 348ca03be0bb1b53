"""Functional regression metrics (parity: reference ``F/regression/__init__.py``)."""
from torchmetrics_amd.functional.regression.correlation import (
    concordance_corrcoef,
    cosine_similarity,
    kendall_rank_corrcoef,
    kl_divergence,
    pearson_corrcoef,
    spearman_corrcoef,
)
from torchmetrics_amd.functional.regression.streaming import (
    critical_success_index,
    explained_variance,
    log_cosh_error,
    mean_absolute_error,
    mean_absolute_percentage_error,
    mean_squared_error,
    mean_squared_log_error,
    minkowski_distance,
    r2_score,
    relative_squared_error,
    symmetric_mean_absolute_percentage_error,
    tweedie_deviance_score,
    weighted_mean_absolute_percentage_error,
)

__all__ = [k for k in dir() if not k.startswith("_")]
