"""Nominal association module metrics (parity: reference ``S/nominal/*.py``).

CramersV / TschuprowsT / PearsonsContingencyCoefficient / TheilsU keep a ``[num_classes, num_classes]`` summed
``confmat`` state (one HIP histogram launch per update, out-of-range values flagged on device and raised at
``compute``); FleissKappa keeps the reference's ``cat`` list of per-sample category counts.
"""
from typing import Any, Literal, Optional

import torch
from torch import Tensor

from torchmetrics_amd.functional.nominal import (
    _cramers_v_compute,
    _fleiss_kappa_compute,
    _fleiss_kappa_update,
    _nominal_confmat,
    _nominal_input_validation,
    _pearsons_contingency_coefficient_compute,
    _theils_u_compute,
    _tschuprows_t_compute,
)
from torchmetrics_amd.metric import Metric
from torchmetrics_amd.utilities.data import dim_zero_cat


class _NominalMetric(Metric):
    full_state_update: bool = False
    is_differentiable: bool = False
    higher_is_better: bool = True
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    _has_bias: bool = True

    def __init__(self, num_classes: int, bias_correction: bool = True, nan_strategy: str = "replace",
                 nan_replace_value: Optional[float] = 0.0, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if not isinstance(num_classes, int) or num_classes < 1:
            raise ValueError(f"Argument `num_classes` is expected to be a positive integer, but got {num_classes}")
        self.num_classes = num_classes
        if self._has_bias:
            if not isinstance(bias_correction, bool):
                raise ValueError(f"Argument `bias_correction` is expected to be a bool, but got {bias_correction}.")
            self.bias_correction = bias_correction
        _nominal_input_validation(nan_strategy, nan_replace_value)
        self.nan_strategy = nan_strategy
        self.nan_replace_value = nan_replace_value
        self.add_state("confmat", torch.zeros(num_classes, num_classes), dist_reduce_fx="sum")

    def update(self, preds: Tensor, target: Tensor) -> None:
        flag = self._device_error_buffer(preds.device) if preds.is_cuda else None
        cm = _nominal_confmat(preds, target, self.num_classes, self.nan_strategy, self.nan_replace_value, flag)
        self.confmat += cm.to(self.confmat.dtype)

    def compute(self) -> Tensor:
        self._raise_device_errors()
        return self._stat(self.confmat)

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


class CramersV(_NominalMetric):
    """Cramer's V (``S/nominal/cramers.py:30``)."""

    def _stat(self, cm: Tensor) -> Tensor:
        return _cramers_v_compute(cm, self.bias_correction)


class TschuprowsT(_NominalMetric):
    """Tschuprow's T (``S/nominal/tschuprows.py:30``)."""

    def _stat(self, cm: Tensor) -> Tensor:
        return _tschuprows_t_compute(cm, self.bias_correction)


class PearsonsContingencyCoefficient(_NominalMetric):
    """Pearson's contingency coefficient (``S/nominal/pearson.py:33``)."""

    _has_bias = False

    def __init__(self, num_classes: int, nan_strategy: str = "replace", nan_replace_value: Optional[float] = 0.0,
                 **kwargs: Any) -> None:
        super().__init__(num_classes, True, nan_strategy, nan_replace_value, **kwargs)

    def _stat(self, cm: Tensor) -> Tensor:
        return _pearsons_contingency_coefficient_compute(cm)


class TheilsU(_NominalMetric):
    """Theil's U (``S/nominal/theils_u.py:30``)."""

    _has_bias = False

    def __init__(self, num_classes: int, nan_strategy: str = "replace", nan_replace_value: Optional[float] = 0.0,
                 **kwargs: Any) -> None:
        super().__init__(num_classes, True, nan_strategy, nan_replace_value, **kwargs)

    def _stat(self, cm: Tensor) -> Tensor:
        return _theils_u_compute(cm)


class FleissKappa(Metric):
    """Fleiss' kappa (``S/nominal/fleiss_kappa.py:29``)."""

    full_state_update: bool = False
    is_differentiable: bool = False
    higher_is_better: bool = True
    plot_upper_bound: float = 1.0

    def __init__(self, mode: Literal["counts", "probs"] = "counts", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        if mode not in ["counts", "probs"]:
            raise ValueError("Argument ``mode`` must be one of 'counts' or 'probs'.")
        self.mode = mode
        self.add_state("counts", default=[], dist_reduce_fx="cat")

    def update(self, ratings: Tensor) -> None:
        self.counts.append(_fleiss_kappa_update(ratings, self.mode))

    def compute(self) -> Tensor:
        return _fleiss_kappa_compute(dim_zero_cat(self.counts))

    def plot(self, val: Optional[Any] = None, ax: Optional[Any] = None) -> Any:
        return self._plot(val, ax)


__all__ = ["CramersV", "FleissKappa", "PearsonsContingencyCoefficient", "TheilsU", "TschuprowsT"]
