"""roctx ranges around the metric lifecycle, for ``rocprofv3 --marker-trace``.

Off by default (zero cost: the hot paths test one module-level bool).  ``TORCHMETRICS_AMD_ROCTX=1`` in the environment,
or :func:`enable` at run time, turns on ranges named

* ``tm.update/<Metric>``, ``tm.forward/<Metric>``, ``tm.compute/<Metric>`` (one per call; :class:`Metric`),
* ``tm.collection.compute`` around a whole :class:`MetricCollection` compute,
* ``tm.sync/<n> states`` around one engine sync and ``tm.sync.bucket/<reduction>/<dtype>/<bytes>B`` around each of its
  collectives (``parallel/sync.py``).

The native C++ entry points (``csrc/bindings/fastcall.cpp`` ``NativeUpdate`` / ``NativeForward``) open the same
``tm.update/<Metric>`` / ``tm.forward/<Metric>`` ranges themselves, so a traced run is the production run: the fast
path stays on and its kernel launches show up inside the ranges.

Ranges go to the rocprofiler-sdk roctx library that rocprofv3 intercepts (``librocprofiler-sdk-roctx.so``); if it is
not present, to torch's roctx binding (``torch.cuda.nvtx`` is roctx on ROCm).  Every range is also a
``torch.profiler.record_function`` while a torch profiler is active.

Example::

    TORCHMETRICS_AMD_ROCTX=1 rocprofv3 --marker-trace --kernel-trace --stats -d out -- python3 bench.py --steps 20
"""
import ctypes
import os
from contextlib import contextmanager
from typing import Callable, Iterator, Optional

ENABLED: bool = os.environ.get("TORCHMETRICS_AMD_ROCTX", "0") not in ("0", "", "false", "False")

_push: Optional[Callable[[str], None]] = None
_pop: Optional[Callable[[], None]] = None


def _bind() -> None:
    global _push, _pop
    if _push is not None:
        return
    for path in ("librocprofiler-sdk-roctx.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                 "libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(path)
            push_a, pop_a = lib.roctxRangePushA, lib.roctxRangePop
        except (OSError, AttributeError):
            continue
        push_a.argtypes, push_a.restype = [ctypes.c_char_p], ctypes.c_int
        pop_a.argtypes, pop_a.restype = [], ctypes.c_int
        _push = lambda name, _f=push_a: _f(name.encode())  # noqa: E731
        _pop = lambda _f=pop_a: _f()  # noqa: E731
        return
    import torch

    nv = torch.cuda.nvtx
    _push = lambda name: nv.range_push(name)  # noqa: E731
    _pop = lambda: nv.range_pop()  # noqa: E731


def enable(on: bool = True) -> None:
    """Turn the lifecycle ranges on (or off) for this process."""
    global ENABLED
    ENABLED = bool(on)
    if ENABLED:
        _bind()
    from torchmetrics_amd import ops

    mod = ops._fast_mod
    if mod is not None and hasattr(mod, "set_ranges"):
        mod.set_ranges(ENABLED)  # the native entry points' ranges


def push(name: str) -> None:
    _bind()
    _push(name)  # type: ignore[misc]
    _torch_ranges.append(_record_function_enter(name))


def pop() -> None:
    rf = _torch_ranges.pop() if _torch_ranges else None
    if rf is not None:
        rf.__exit__(None, None, None)
    _pop()  # type: ignore[misc]


_torch_ranges: list = []


def _record_function_enter(name: str):
    """A torch.profiler.record_function entered now, if a torch profiler is collecting (else None)."""
    import torch

    if not torch.autograd._profiler_enabled():
        return None
    rf = torch.profiler.record_function(name)
    rf.__enter__()
    return rf


@contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - the roctx vocabulary
    """``with profiling.range("name"): ...`` -- a roctx range when ranges are on, nothing otherwise."""
    if not ENABLED:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()


if ENABLED:
    _bind()

__all__ = ["ENABLED", "enable", "push", "pop", "range"]
