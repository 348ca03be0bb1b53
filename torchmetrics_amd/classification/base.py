"""Task-wrapper base (parity: reference ``S/classification/base.py:19-32``).

``Accuracy(task="multiclass", ...)`` etc. are factories: ``__new__`` returns the concrete task class, so the wrapper
itself is never updated or computed.
"""
from typing import Any

from torchmetrics_amd.metric import Metric


class _ClassificationTaskWrapper(Metric):
    def update(self, *args: Any, **kwargs: Any) -> None:
        raise NotImplementedError(
            f"{self.__class__.__name__} metric does not have a global `update` method. Use the task specific metric."
        )

    def compute(self) -> None:
        raise NotImplementedError(
            f"{self.__class__.__name__} metric does not have a global `compute` method. Use the task specific metric."
        )
