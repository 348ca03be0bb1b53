"""Host-side warnings that depend on a device value, made capturable.

A few computes warn on a device condition (e.g. "AUROC of a class was nan", reference
``F/classification/average_precision.py`` / ``auroc.py`` ``_reduce_average``): reading the flag is a device sync, which
a HIP graph cannot contain.  :func:`warn_if` reads the flag eagerly, but while a :class:`capture_sink` is active on a
capturing stream it records ``(flag, message)`` instead; :class:`torchmetrics_amd.utils.graphs.GraphedCompute` then
reads those flags together with the validation words (one device->host copy per replay) and warns after the replay.
"""
from typing import List, Optional, Tuple, Type

import torch
from torch import Tensor

from torchmetrics_amd.utilities.prints import rank_zero_warn

_SINK: Optional[List[Tuple[Tensor, str, Optional[Type[Exception]]]]] = None
_SUPPRESS = False


class suppress:  # noqa: N801 - context manager
    """Skip the checks entirely (warm-up runs on states that may not hold data yet)."""

    def __enter__(self) -> "suppress":
        global _SUPPRESS
        self._prev = _SUPPRESS
        _SUPPRESS = True
        return self

    def __exit__(self, *exc) -> None:
        global _SUPPRESS
        _SUPPRESS = self._prev


class capture_sink:  # noqa: N801 - context manager
    def __init__(self) -> None:
        self.items: List[Tuple[Tensor, str, Optional[Type[Exception]]]] = []

    def __enter__(self) -> "capture_sink":
        global _SINK
        self._prev = _SINK
        _SINK = self.items
        return self

    def __exit__(self, *exc) -> None:
        global _SINK
        _SINK = self._prev


def warn_if(flag: Tensor, message: str) -> None:
    """``rank_zero_warn(message)`` if ``flag`` (any shape; any non-zero element) is set."""
    if _SUPPRESS:
        return
    if _SINK is not None and flag.is_cuda and torch.cuda.is_current_stream_capturing():
        _SINK.append((flag, message, None))
        return
    if bool(flag.any()):
        rank_zero_warn(message, UserWarning)


def raise_if(cond: Tensor, exc_type: Type[Exception], message: str) -> None:
    """``raise exc_type(message)`` if ``cond`` is set; under a graph capture the check runs after each replay."""
    if _SUPPRESS:
        return
    if not isinstance(cond, Tensor):
        if cond:
            raise exc_type(message)
        return
    if _SINK is not None and cond.is_cuda and torch.cuda.is_current_stream_capturing():
        _SINK.append((cond, message, exc_type))
        return
    if bool(cond.any()):
        raise exc_type(message)


__all__ = ["warn_if", "raise_if", "capture_sink", "suppress"]
