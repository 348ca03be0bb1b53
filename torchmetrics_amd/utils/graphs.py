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
import warnings
from typing import Any, Dict, List, Optional, Tuple, Union

import torch
import torch.distributed as dist
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.collections import MetricCollection
from torchmetrics_amd.metric import CompositionalMetric, Metric
from torchmetrics_amd.parallel import arena as _arena
from torchmetrics_amd.parallel import sync as _sync
from torchmetrics_amd.utilities.data import _squeeze_if_scalar
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils.deferred import WORD_CODES, capture_sink
from torchmetrics_amd.utils.deferred import suppress as suppress_checks


class UpdateGroup:
    """Several metrics / collections fed from different inputs, updated together: ``UpdateGroup((cls, 2), (reg, 2))``
    takes ``update(logits, labels, x, y)`` and hands the first two inputs to ``cls``, the next two to ``reg``.  With
    :class:`GraphedUpdate` the whole group replays from ONE graph (a ``hipGraphLaunch`` costs ~15-30 us of host time on
    ROCm, so one launch per step instead of one per collection)."""

    def __init__(self, *parts: Tuple[Union[Metric, MetricCollection], int]) -> None:
        self.parts = [(t, int(n)) for t, n in parts]

    def update(self, *inputs: Tensor) -> None:
        pos = 0
        for t, n in self.parts:
            t.update(*inputs[pos : pos + n])
            pos += n

    def reset(self) -> None:
        for t, _ in self.parts:
            t.reset()


def _members(target: Union[Metric, MetricCollection, UpdateGroup]) -> List[Tuple[str, Metric]]:
    if isinstance(target, UpdateGroup):
        return [(f"{i}:{n}", m) for i, (t, _) in enumerate(target.parts) for n, m in _members(t)]
    if isinstance(target, MetricCollection):
        return list(target.items(keep_base=True, copy_state=False))
    return [(type(target).__name__, target)]


def _states(metrics: List[Tuple[str, Metric]]) -> Dict[Tuple[str, str], Any]:
    return {(name, attr): getattr(m, attr) for name, m in metrics for attr in m._defaults}


class GraphedUpdate:
    """``GraphedUpdate(metric_or_collection, *example_inputs)``; then call it with each batch instead of ``update``."""

    def __init__(self, target: Union[Metric, MetricCollection, UpdateGroup], *example_inputs: Tensor, warmup: int = 2,
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


# ------------------------------------------------------------------------------------------------------ compute
def _leaves(obj: Any, out: List[Tensor]) -> Any:
    """Replace every tensor of a (nested dict / list / tuple) result by its index in ``out``."""
    if isinstance(obj, Tensor):
        out.append(obj)
        return ("__leaf__", len(out) - 1)
    if isinstance(obj, dict):
        return {k: _leaves(v, out) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_leaves(v, out) for v in obj)
    return obj


def _rebuild(spec: Any, leaves: List[Tensor]) -> Any:
    if isinstance(spec, tuple) and len(spec) == 2 and spec[0] == "__leaf__":
        return leaves[spec[1]]
    if isinstance(spec, dict):
        return {k: _rebuild(v, leaves) for k, v in spec.items()}
    if isinstance(spec, (list, tuple)):
        return type(spec)(_rebuild(v, leaves) for v in spec)
    return spec


def _same_result(a: Any, b: Any) -> bool:
    if isinstance(a, Tensor):
        return isinstance(b, Tensor) and a.shape == b.shape and a.dtype == b.dtype and bool(
            torch.equal(a, b) or torch.allclose(a, b, rtol=0, atol=0, equal_nan=True))
    if isinstance(a, dict):
        return isinstance(b, dict) and a.keys() == b.keys() and all(_same_result(a[k], b[k]) for k in a)
    if isinstance(a, (list, tuple)):
        return isinstance(b, (list, tuple)) and len(a) == len(b) and all(_same_result(x, y) for x, y in zip(a, b))
    return a == b


def _contig_strides(shape: Tuple[int, ...]) -> Tuple[int, ...]:
    st, acc = [], 1
    for d in reversed(shape):
        st.append(acc)
        acc *= d
    return tuple(reversed(st))


_WORD_CODES = WORD_CODES


class GraphedCompute:
    """``compute()`` of a metric or collection with the tensor-state members replayed from ONE HIP graph.

    The graph holds, per call: the one-block reductions of the stat-score / confusion-matrix / binned-curve /
    streaming-regression members, recorded as tasks and run by ONE kernel (``ops.fused_compute``,
    ``csrc/common/compute_tasks.hip``; a member joins only if its recorded compute reproduces its eager result bit for
    bit at capture time), the remaining ops of members that are not fused, and one kernel that writes every member's
    deferred-validation word and device-side warning flag into pinned host memory.  After the replay the results are
    copied out of the graph's static outputs (one ``cat`` per dtype) and the status words are read with no copy: a bad
    batch still raises, with the member's own message.  Members with list states, custom sync functions or computes
    that cannot be captured (host syncs) run through their normal ``compute()``.

    Under ``torch.distributed`` the graph reads a persistent arena instead of the live states: each call copies the
    states into it (one copy of the members' packed state arena per (reduction, dtype) bucket, ``parallel/arena.py``;
    a ``torch.cat(out=)`` if a state fell out of it) and all-reduces the buckets in place (the
    engine's one-shot xGMI kernel for small buckets, RCCL otherwise -- the reduction ``sync()`` would apply).  On one
    process the graph reads the live states; ``reset()`` / ``load_state_dict`` rebinding them triggers a re-capture.

    Results equal ``target.compute()``; local states are never modified (sync + compute + unsync semantics).
    The graph bakes the members' Python configuration (``average``, ``num_classes`` ...) and the state shapes at
    capture: after changing either, call :meth:`recapture`.

    Reference: the sync / compute sequence this replaces is ``S/collections.py:310-359`` + ``S/metric.py:427-457``.
    """

    def __init__(self, *targets: Union[Metric, MetricCollection]) -> None:
        if not targets:
            raise ValueError("GraphedCompute needs at least one metric or collection")
        self.targets = targets
        self.target = targets[0]
        self._force_arena = False
        self._rebinds = 0
        self._capture()

    # ---------------------------------------------------------------------------------------------- capture
    @staticmethod
    def _world(m: Metric) -> int:
        if not _sync.distributed_available():
            return 1
        return dist.get_world_size(m.process_group)

    def _graphable(self, m: Metric) -> Optional[str]:
        """None if ``m`` can be replayed, else the reason it stays eager."""
        if isinstance(m, CompositionalMetric) or not isinstance(m, Metric) or not m._defaults:
            return "not a plain metric with states"
        for a in m._defaults:
            v = getattr(m, a)
            if not isinstance(v, Tensor):
                return f"list state `{a}`"
            if not v.is_cuda:
                return f"state `{a}` is not on a ROCm device"
        if self._world(m) > 1:
            if m.dist_sync_fn is not None or type(m)._sync_dist is not Metric._sync_dist or not m._to_sync:
                return "custom or disabled sync"
            if m.process_group is not None:
                return "process-group subset"
            if any(_sync._reduce_kind(m._reductions[a]) is None for a in m._defaults):
                return "state without a sum/mean/max/min reduction"
        return None

    def _capture(self) -> None:
        self._capture_errors: Dict[str, str] = {}
        self._probed: set = set()
        self._fusable: set = set()
        # several targets share one graph (one replay, one status read); member names are made unique per target
        members = []
        self._owner: Dict[str, Tuple[int, str]] = {}
        for ti, t in enumerate(self.targets):
            for n, m in _members(t):
                key = n if len(self.targets) == 1 else f"{ti}:{n}"
                self._owner[key] = (ti, n)
                members.append((key, m))
        self._all_members = members
        cand = []
        for n, m in members:
            why = self._graphable(m)
            if why is None:
                cand.append((n, m))
            else:
                self._capture_errors[n] = why
        self._world_size = max([self._world(m) for _, m in cand] or [1])
        good: List[Tuple[str, Metric]] = []
        for n, m in cand:  # a member whose compute cannot be captured (host sync ...) stays eager
            if self._try_capture([(n, m)]) is not None:
                good.append((n, m))
        self._graphed = good
        self._graph = self._try_capture(good) if good else None
        if good and self._graph is None:
            raise RuntimeError(f"GraphedCompute: capture of the combined graph failed: {self._capture_errors}")
        graphed = {n for n, _ in good}
        self._eager = [(n, m) for n, m in members if n not in graphed]
        self._keys = self._output_keys()

    def _output_keys(self) -> Optional[Dict[str, str]]:
        """member -> output key when every target is a collection of plain-valued members (no dict results to
        flatten), else None."""
        for t in self.targets:
            if not isinstance(t, MetricCollection):
                return None
        for _, m in self._all_members:
            if getattr(m, "_from_collection", None):
                return None
        return {key: self.targets[ti]._set_name(n) for key, (ti, n) in self._owner.items()}

    def _try_capture(self, members: List[Tuple[str, Metric]]) -> Optional[torch.cuda.CUDAGraph]:
        use_arena = self._world_size > 1 or self._force_arena
        if use_arena and self._world_size > 1:
            # lay the live states out in this graph's bucket order (parallel/arena.py): each replay then copies every
            # bucket with ONE copy of its span
            self._pack_live(members)
        # distinct live state tensors, bucketed by (reduction, dtype) for the arena
        buckets: Dict[Tuple[str, torch.dtype], List[Tuple[Metric, str, Tensor]]] = {}
        seen: Dict[int, Tuple[str, torch.dtype]] = {}
        uses: List[Tuple[Metric, str, Tensor]] = []
        for _, m in members:
            for a in m._defaults:
                t = getattr(m, a)
                uses.append((m, a, t))
                if id(t) in seen:
                    continue
                key = (_sync._reduce_kind(m._reductions[a]) or "none", t.dtype)
                seen[id(t)] = key
                buckets.setdefault(key, []).append((m, a, t))
        arenas: Dict[Tuple[str, torch.dtype], Tensor] = {}
        views: Dict[int, Tensor] = {}
        if use_arena:
            for key, items in buckets.items():
                flat = torch.empty(sum(t.numel() for _, _, t in items), dtype=key[1], device=items[0][2].device)
                off = 0
                for _, _, t in items:
                    views[id(t)] = flat[off : off + t.numel()].view(t.shape)
                    off += t.numel()
                arenas[key] = flat
        # the one-shot buckets' status word (replays all-reduce the arena BEFORE the graph runs; allocated here, outside
        # the capture, so no captured memset clears it): the graph gathers it with the validation words, and one host
        # read after the replay sees a failed bucket
        oneshot_word: Optional[Tensor] = None
        if use_arena and self._world_size > 1 and arenas:
            oneshot_word = torch.zeros(1, dtype=torch.int32, device=next(iter(arenas.values())).device)
        words = [(m._device_errors, 0) for _, m in self._all_members
                 if m._device_errors is not None and m._device_errors.is_cuda]
        graph = torch.cuda.CUDAGraph()
        probe = len(members) == 1 and members[0][0] not in self._probed
        host_words = torch.zeros(128, dtype=torch.int32, pin_memory=True)
        host_ptr = int(ops._ops().mapped_device_ptr(host_words))
        try:
            if use_arena:
                for key, items in buckets.items():
                    torch.cat([t.reshape(-1) for _, _, t in items], out=arenas[key])
                for m, a, t in uses:
                    m.__dict__[a] = views[id(t)]
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            # warm-up (lazily created workspaces reach their steady state); the metrics' data checks are skipped:
            # the states may not hold enough data yet, and inside the graph they run after every replay
            with torch.cuda.stream(side), suppress_checks(), warnings.catch_warnings():
                warnings.simplefilter("ignore")
                eager = [type(m).compute(m) for _, m in members]
                if probe:
                    # can this member's reductions join the one-launch task kernel?  Run it recorded, with the
                    # outputs poisoned until the flush: a consumer that reads an output before the flush (anything
                    # but a view) would see the poison and the results would differ from the eager ones
                    with ops.fused_compute(poison=True) as rec:
                        recorded = type(members[0][1]).compute(members[0][1])
                    n_tasks = rec.flush()
            torch.cuda.current_stream().wait_stream(side)
            if probe:
                self._probed.add(members[0][0])
                if n_tasks and _same_result(eager[0], recorded):
                    self._fusable.add(members[0][0])
            leaves: List[Tensor] = []
            with capture_sink() as sink, torch.cuda.graph(graph):
                results = {}
                for n, m in members:
                    if probe or n not in self._fusable:
                        results[n] = type(m).compute(m)
                with ops.fused_compute() as rec:
                    for n, m in members:
                        if not probe and n in self._fusable:
                            results[n] = type(m).compute(m)
                rec.flush()
                spec = [_leaves(_squeeze_if_scalar(results[n]), leaves) for n, _ in members]
                # every result leaf of one dtype lands in one static buffer: a replay's results are ONE copy per dtype
                by_dtype: Dict[torch.dtype, List[int]] = {}
                for i, t in enumerate(leaves):
                    by_dtype.setdefault(t.dtype, []).append(i)
                outs = {dt: torch.cat([leaves[i].reshape(-1) for i in idx]) for dt, idx in by_dtype.items()}
                # validation words + device-side warning conditions -> pinned host memory, one kernel
                for f, _, _ in sink.items:
                    flat = f.reshape(-1)
                    if flat.numel() != 1 or flat.dtype not in _WORD_CODES:
                        flat = flat.to(torch.int32).amax().reshape(1)
                    words.append((flat, _WORD_CODES[flat.dtype]))
                if oneshot_word is not None:
                    words.append((oneshot_word, 0))  # gathered last (see its allocation above)
                if len(words) > host_words.numel():
                    raise RuntimeError("GraphedCompute: more than 128 status words")
                if words:
                    table = torch.tensor([[w.data_ptr(), c] for w, c in words], dtype=torch.int64)
                    ops._ops().gather_words(table, host_ptr, words[0][0])
        except Exception as err:  # noqa: BLE001 - not capturable: the caller keeps the member(s) eager
            torch.cuda.synchronize()
            self._capture_errors[",".join(n for n, _ in members)] = repr(err)
            return None
        finally:
            if use_arena:
                for m, a, t in uses:
                    m.__dict__[a] = t
        self._use_arena = use_arena
        self._buckets = [(key, [(m, a) for m, a, _ in items], arenas[key]) for key, items in buckets.items()
                         if key in arenas]
        self._uses = uses
        self._spec = spec
        self._outs = outs
        self._leaf_views = []  # (dtype, shape, offset) per leaf, into its dtype's buffer
        self._n_leaves = len(leaves)
        for dt, idx in by_dtype.items():
            off = 0
            for i in idx:
                self._leaf_views.append((i, dt, tuple(leaves[i].shape), off))
                off += leaves[i].numel()
        self._host_words = host_words[: len(words)] if words else None
        self._oneshot_word = oneshot_word
        self._word_keep = words  # the flag tensors the graph reads
        self._err_members = [m for _, m in self._all_members if m._device_errors is not None and m._device_errors.is_cuda]
        self._n_err = len(self._err_members)
        self._checks = [(msg, exc) for _, msg, exc in sink.items]
        self._err_ids = {id(m._device_errors) for m in self._err_members}
        return graph

    def _pack_live(self, members: List[Tuple[str, Metric]]) -> None:
        seen: set = set()
        buckets: Dict[Tuple[str, torch.dtype], List[Tuple[Metric, str, Tensor]]] = {}
        for _, m in members:
            for a in m._defaults:
                t = getattr(m, a)
                if id(t) in seen or not isinstance(t, Tensor):
                    continue
                seen.add(id(t))
                kind = _sync._reduce_kind(m._reductions[a])
                if kind is not None:
                    buckets.setdefault((kind, t.dtype), []).append((m, a, t))
        moved = False
        for items in buckets.values():
            if len(items) > 1 and _arena.contiguous_span([t for _, _, t in items]) is None:
                _arena.pack_items(items)
                moved = True
        if moved:
            for t in self.targets:
                if isinstance(t, MetricCollection):
                    t._compute_groups_create_state_ref()  # compute-group followers see the packed views

    def recapture(self) -> None:
        self._capture()

    # ------------------------------------------------------------------------------------------------- replay
    def _stale(self) -> bool:
        for _, m in self._all_members:
            e = m.__dict__.get("_device_errors")
            if e is not None and e.is_cuda and id(e) not in self._err_ids:
                return True  # a validation word was (re)created after capture
        if not self._use_arena:
            for m, a, t in self._uses:
                if m.__dict__.get(a) is not t:
                    # reset() / load_state_dict / .to() rebound a state the graph reads; a member whose update
                    # rebinds its states every time makes the graph read a packed arena instead
                    self._rebinds += 1
                    if self._rebinds >= 3:
                        self._force_arena = True
                    return True
        return False

    def _replay(self) -> Dict[str, Any]:
        if self._use_arena:
            for _, pairs, flat in self._buckets:
                live = [getattr(m, a) for m, a in pairs]
                span = _arena.contiguous_span(live)
                if span is not None:
                    flat.copy_(span)  # the members' packed arena (parallel/arena.py): one copy
                else:
                    torch.cat([t.reshape(-1) for t in live], out=flat)
            for (kind, _dt), _, flat in self._buckets:
                if kind == "none":
                    continue
                comm = _sync.get_oneshot(None) if _sync._is_nccl(None) else None
                if comm is not None and comm.supports(flat):
                    word = self._oneshot_word
                    comm.all_reduce(flat, kind, word if word is not None and word.device == flat.device else None)
                else:
                    _sync._all_reduce(flat, kind, None)
                if kind == "mean":
                    flat.div_(self._world_size)
        self._graph.replay()
        copies = {dt: buf.clone() for dt, buf in self._outs.items()}  # fresh results: one copy per dtype
        leaves: List[Optional[Tensor]] = [None] * self._n_leaves
        strided = torch.as_strided
        for i, dt, shape, off in self._leaf_views:
            leaves[i] = strided(copies[dt], shape, _contig_strides(shape), off)
        if self._host_words is not None:
            torch.cuda.current_stream().synchronize()
            codes = self._host_words.tolist()
            if self._oneshot_word is not None and codes[-1]:
                self._oneshot_word.zero_()
                from torchmetrics_amd.utils import validation as _validation

                _validation.raise_for_code(codes[-1])  # never hand out values from a failed sync
            if any(codes):
                ne = self._n_err
                for m, code in zip(self._err_members, codes[:ne]):
                    if code:
                        m.__dict__["_device_errors"].zero_()
                        from torchmetrics_amd.utils import validation as _validation

                        _validation.raise_for_code(code, m)
                for (msg, exc), code in zip(self._checks, codes[ne:]):
                    if code and exc is not None:
                        raise exc(msg)
                for (msg, exc), code in zip(self._checks, codes[ne:]):
                    if code:
                        rank_zero_warn(msg, UserWarning)
        return {n: _rebuild(spec, leaves) for (n, _), spec in zip(self._graphed, self._spec)}

    def _eager_all(self) -> Any:
        outs = [t.compute() for t in self.targets]
        return outs[0] if len(outs) == 1 else tuple(outs)

    def __call__(self) -> Any:
        """The targets' ``compute()`` results (a tuple of them when several targets were given)."""
        if self._graph is None:
            return self._eager_all()
        for t in self.targets:
            if isinstance(t, MetricCollection):
                t._compute_groups_create_state_ref()  # group members see their leader's current states
        if self._stale():
            self._capture()
            if self._graph is None:
                return self._eager_all()
        results = self._replay()
        for _, m in self._all_members:
            d = m.__dict__
            if d["_device_errors"] is not None:
                d["_errors_checked_at"] = d["_update_count"]  # read clean just now
        keys = self._keys
        if keys is not None:
            # plain per-member values: build the collections' outputs directly
            outs: List[Dict[str, Any]] = [{} for _ in self.targets]
            for n, m in self._all_members:
                ti = self._owner[n][0]
                if n in results:
                    if m.__dict__["_update_count"] == 0:
                        rank_zero_warn(f"The ``compute`` method of metric {m.__class__.__name__} was called before "
                                       "the ``update`` method which may lead to errors, as metric states have not "
                                       "yet been updated.", UserWarning)
                    outs[ti][keys[n]] = results[n]
                else:
                    outs[ti][keys[n]] = m.compute()
            return outs[0] if len(outs) == 1 else tuple(outs)
        marks = []
        for n, m in self._all_members:
            if n in results:
                d = m.__dict__
                marks.append((d, d["_computed"]))
                d["_computed"] = results[n]
        try:
            return self._eager_all()
        finally:
            for d, prev in marks:
                if not d["compute_with_cache"]:
                    d["_computed"] = prev


__all__ = ["GraphedUpdate", "GraphedCompute", "UpdateGroup"]
