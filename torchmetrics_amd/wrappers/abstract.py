"""Base for wrapper metrics (parity: reference ``S/wrappers/abstract.py:19-42``).

A wrapper delegates sync/caching to the wrapped metric, so the update/compute wrapping is disabled.
"""
from typing import Any, Callable

from torchmetrics_amd.metric import Metric


class WrapperMetric(Metric):
    def _wrap_update(self, update: Callable) -> Callable:
        return update

    def _wrap_compute(self, compute: Callable) -> Callable:
        return compute

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        raise NotImplementedError
