"""Host-side warnings that depend on a device value, made capturable.

A few computes warn on a device condition (e.g. "AUROC of a class was nan", reference
``F/classification/average_precision.py`` / ``auroc.py`` ``_reduce_average``): reading the flag is a device sync, which
a HIP graph cannot contain.  :func:`warn_if` reads the flag eagerly, but while a :class:`capture_sink` is active on a
capturing stream it records ``(flag, message)`` instead; :class:`torchmetrics_amd.utils.graphs.GraphedCompute` then
reads those flags together with the validation words (one device->host copy per replay) and warns after the replay.
Under :class:`defer` (eager) the flags are collected the same way and read once by their owner.
"""
from typing import List, Optional, Tuple, Type

import torch
from torch import Tensor

from torchmetrics_amd.utilities.prints import rank_zero_warn

_SINK: Optional[List[Tuple[Tensor, str, Optional[Type[Exception]]]]] = None
_SUPPRESS = False
# dtype -> code of ops.gather_words (the kernel reads element 0 of a word as int32 / f32 / f64 / i64 / byte)
WORD_CODES = {torch.int32: 0, torch.float32: 1, torch.float64: 2, torch.int64: 3, torch.uint8: 4, torch.bool: 4}
# eager deferral (a MetricCollection's compute(): every member's checks are read with ONE device read at the end)
_DEFER: Optional[List[Tuple[Tensor, str, Optional[Type[Exception]]]]] = None


class defer:  # noqa: N801 - context manager
    """Collect the device-side checks of eager code instead of reading each one (a device sync per check); the owner
    reads the collected flags together (:meth:`MetricCollection.compute` folds them into its one status read) and then
    raises / warns in recording order.  Multi-element flags are reduced on the device (one ``any``) when recorded."""

    def __init__(self) -> None:
        self.items: List[Tuple[Tensor, str, Optional[Type[Exception]]]] = []

    def __enter__(self) -> "defer":
        global _DEFER
        self._prev = _DEFER
        _DEFER = self.items
        return self

    def __exit__(self, *exc) -> None:
        global _DEFER
        _DEFER = self._prev


def _record(flag: Tensor, message: str, exc_type: Optional[Type[Exception]]) -> bool:
    if _SINK is not None and flag.is_cuda and torch.cuda.is_current_stream_capturing():
        _SINK.append((flag, message, exc_type))
        return True
    if _DEFER is not None and flag.is_cuda:
        _DEFER.append((flag if flag.numel() == 1 else flag.any(), message, exc_type))
        return True
    return False


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
    if _SUPPRESS or _record(flag, message, None):
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
    if _record(cond, message, exc_type):
        return
    if bool(cond.any()):
        raise exc_type(message)


__all__ = ["warn_if", "raise_if", "capture_sink", "suppress", "defer", "WORD_CODES"]
