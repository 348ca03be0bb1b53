"""HIP-graph capture of ``update`` for fixed-shape evaluation loops.

A metric ``update`` on MI355X is a handful of short kernels; with a whole ``MetricCollection`` the host-side Python
and launch work per step (tens of µs) exceeds the GPU time.  :class:`GraphedUpdate` records ``target.update`` once
into a HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replays it for each new batch: the replay is one
graph launch plus one device copy per input, whatever the number of metrics and kernels.

Constraints (checked at capture):

* every state is a tensor updated in place -- list ("cat") states grow by appending new tensors and cannot be
  replayed (``MulticlassCalibrationError``, unbinned curves, retrieval ...): keep those metrics eager;
* the update must not rebind a state to a new tensor object, nor synchronise with the host;
* inputs keep the example's shapes / dtypes (a new shape needs a new capture).

By default the example inputs are cloned into private static buffers and every call copies the new batch in (one
device copy per input).  With ``bind_inputs=True`` the graph reads the example tensors themselves: a producer that
writes each batch into those tensors (a model writing ``out=``, a pinned-memory ring filled by the data loader) calls
the graph with them -- or with no arguments -- and no copy is made.  A ring of N input buffers is served by N
``GraphedUpdate(..., bind_inputs=True)`` objects over the same target, one per buffer.

The metric's Python bookkeeping (``update_count``, the ``compute`` cache) is advanced on every replay, so
``compute()``, ``reset()``, sync and ``state_dict`` behave exactly as after eager updates.  ``reset()`` re-creates the
state tensors: the next call notices (one identity check per member) and re-captures before replaying.
"""
from typing import Any, Dict, List, Tuple, Union

import torch
from torch import Tensor

from torchmetrics_amd.collections import MetricCollection
from torchmetrics_amd.metric import Metric


def _members(target: Union[Metric, MetricCollection]) -> List[Tuple[str, Metric]]:
    if isinstance(target, MetricCollection):
        return list(target.items(keep_base=True, copy_state=False))
    return [(type(target).__name__, target)]


def _states(metrics: List[Tuple[str, Metric]]) -> Dict[Tuple[str, str], Any]:
    return {(name, attr): getattr(m, attr) for name, m in metrics for attr in m._defaults}


class GraphedUpdate:
    """``GraphedUpdate(metric_or_collection, *example_inputs)``; then call it with each batch instead of ``update``."""

    def __init__(self, target: Union[Metric, MetricCollection], *example_inputs: Tensor, warmup: int = 2,
                 bind_inputs: bool = False) -> None:
        if not example_inputs or not all(isinstance(a, Tensor) and a.is_cuda for a in example_inputs):
            raise ValueError("GraphedUpdate needs the example inputs as ROCm tensors")
        self.target = target
        self._members = _members(target)
        for name, m in self._members:
            for attr in m._defaults:
                if not isinstance(getattr(m, attr), Tensor):
                    raise ValueError(f"metric `{name}` has the list state `{attr}`: it cannot be replayed from a graph")
        self._static = [a.detach() if bind_inputs else a.detach().clone() for a in example_inputs]
        self._bound = bind_inputs
        self._warmup = warmup
        self._capture()

    def _capture(self) -> None:
        members = self._members
        counts = {name: m._update_count for name, m in members}
        # warm up on a side stream (workspaces, compute groups, lazily-created buffers reach their steady state)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        snapshot = None
        # the warm-up runs on the example buffers, which may hold garbage (bound producer buffers are often
        # torch.empty at capture time): the validation words are restored with the states afterwards
        errs = {name: (m._device_errors.clone() if m._device_errors is not None else None) for name, m in members}
        with torch.cuda.stream(side):
            for _ in range(max(self._warmup, 1)):
                before = _states(members)
                if snapshot is None:
                    snapshot = {k: v.clone() for k, v in before.items()}
                self.target.update(*self._static)
        torch.cuda.current_stream().wait_stream(side)
        before = _states(members)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.target.update(*self._static)
        after = _states(members)
        rebound = [f"{n}.{a}" for (n, a), t in after.items() if t is not before[(n, a)]]
        if rebound:
            raise RuntimeError(f"update() rebinds states {rebound}: not capturable, keep these metrics eager")
        # undo the warm-up updates: the captured graph has not executed yet
        with torch.no_grad():
            for key, val in _states(members).items():
                val.copy_(snapshot[key] if key in snapshot else val)
        for name, m in members:
            m.__dict__["_update_count"] = counts[name]
            m.__dict__["_computed"] = None
            m.__dict__.pop("_errors_checked_at", None)
            buf = m._device_errors
            if buf is not None:
                if errs[name] is None:
                    buf.zero_()
                else:
                    buf.copy_(errs[name])
        # one state tensor per member: a replay checks these are still the metric's states (reset() rebinds them)
        self._sentinels = [(m, attr, after[(name, attr)]) for name, m in members
                           for attr in list(m._defaults)[:1]]

    def recapture(self) -> None:
        """Capture again (after ``reset()`` re-created the state tensors, or after moving the metric)."""
        self._capture()

    def __call__(self, *inputs: Tensor) -> None:
        if not inputs and self._bound:
            inputs = tuple(self._static)  # the producer already wrote the bound buffers
        if len(inputs) != len(self._static):
            raise ValueError(f"expected {len(self._static)} inputs, got {len(inputs)}")
        for s, x in zip(self._static, inputs):
            if x is s or (x.data_ptr() == s.data_ptr() and x.shape == s.shape and x.stride() == s.stride()
                          and x.dtype == s.dtype):
                continue  # the captured buffer itself: nothing to copy
            if x.shape != s.shape or x.dtype != s.dtype:
                raise ValueError(f"input of shape {tuple(x.shape)} / {x.dtype} does not match the captured "
                                 f"{tuple(s.shape)} / {s.dtype}; capture a new GraphedUpdate for it")
            s.copy_(x, non_blocking=True)
        for m, attr, t in self._sentinels:
            if m.__dict__.get(attr) is not t and getattr(m, attr) is not t:
                # reset() / load_state_dict / .to() rebound the states: the graph would replay into orphaned tensors
                self._capture()
                break
        self.graph.replay()
        for _, m in self._members:
            d = m.__dict__
            d["_update_count"] += 1
            d["_computed"] = None


__all__ = ["GraphedUpdate"]
