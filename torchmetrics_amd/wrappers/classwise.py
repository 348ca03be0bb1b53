"""Per-class dict output for metrics with ``average=None`` (reference ``S/wrappers/classwise.py:26-200``).

The output keys depend only on the configuration and the number of classes, so they are built once per class count
and reused: ``compute()`` is one ``unbind`` of the wrapped result plus a ``dict(zip(...))``.
"""
from typing import Any, Dict, List, Optional, Tuple

from torch import Tensor

from torchmetrics_amd.metric import Metric
from torchmetrics_amd.wrappers.abstract import WrapperMetric


def _check_optional(value: Any, ok: bool, name: str, what: str) -> None:
    if value is not None and not ok:
        raise ValueError(f"Expected argument `{name}` to either be `None` or {what} but got {value}")


class ClasswiseWrapper(WrapperMetric):
    """Turn a per-class tensor result into ``{prefix + label + postfix: value}``."""

    def __init__(
        self,
        metric: Metric,
        labels: Optional[List[str]] = None,
        prefix: Optional[str] = None,
        postfix: Optional[str] = None,
    ) -> None:
        super().__init__()
        if not isinstance(metric, Metric):
            raise ValueError(f"Expected argument `metric` to be an instance of `torchmetrics.Metric` but got {metric}")
        _check_optional(labels, isinstance(labels, list) and all(isinstance(s, str) for s in labels),
                        "labels", "a list of strings")
        _check_optional(prefix, isinstance(prefix, str), "prefix", "a string")
        _check_optional(postfix, isinstance(postfix, str), "postfix", "a string")
        self.metric = metric
        self.labels = labels
        self._prefix = prefix
        self._postfix = postfix
        self._keys: Tuple[Any, List[str]] = (None, [])
        self._update_count = 1

    def _names(self, n: int) -> List[str]:
        key = (n, None if self.labels is None else tuple(self.labels), self._prefix, self._postfix)
        if self._keys[0] != key:
            # no prefix and no postfix: "<metric class name>_" in front (the reference's default naming)
            if self._prefix or self._postfix:
                head, tail = self._prefix or "", self._postfix or ""
            else:
                head, tail = type(self.metric).__name__.lower() + "_", ""
            labels = list(range(n)) if self.labels is None else self.labels
            self._keys = (key, [f"{head}{lab}{tail}" for lab in labels])
        return self._keys[1]

    def _convert(self, x: Tensor) -> Dict[str, Any]:
        return dict(zip(self._names(len(x)), x))

    def forward(self, *args: Any, **kwargs: Any) -> Any:
        return self._convert(self.metric(*args, **kwargs))

    def update(self, *args: Any, **kwargs: Any) -> None:
        self.metric.update(*args, **kwargs)

    def compute(self) -> Dict[str, Tensor]:
        return self._convert(self.metric.compute())

    def reset(self) -> None:
        self.metric.reset()
