"""Core runtime: the ``Metric`` base class and ``CompositionalMetric``.

Lifecycle parity with reference ``S/metric.py:50-1211`` (``add_state`` / ``update`` / ``compute`` / ``forward`` /
``reset`` / ``sync`` / ``unsync`` / ``sync_context`` / ``state_dict`` / pickling / operator algebra).

MI355X-first differences:

* **Sync** (``_sync_dist``): with ``dist_sync_fn=None`` (the default) states go through the bucketed engine in
  :mod:`torchmetrics_amd.parallel.sync` -- one RCCL ``all_reduce`` per (op, dtype) bucket for SUM/MEAN/MAX/MIN states,
  one packed ``all_gather`` per dtype for CAT/None states, no barriers.  A user-supplied ``dist_sync_fn`` keeps the
  reference per-tensor contract exactly (``fn(tensor, group=...) -> List[Tensor]``, ``T/bases/test_metric.py:517``).
* **Deferred validation**: HIP kernels validate value ranges on device and raise bits in ``self._device_errors``;
  the flags are read once (a 4-byte D2H copy) at ``compute()`` instead of the reference's per-``update`` host syncs
  (``F/classification/stat_scores.py:307,316``).  ``TORCHMETRICS_AMD_STRICT=1`` checks after every update.
"""
import builtins
import functools
import inspect
import sys
from abc import ABC, abstractmethod
from contextlib import contextmanager, nullcontext
from copy import deepcopy
from typing import Any, Callable, Dict, Generator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module, Parameter

from torchmetrics_amd import ops as _ops
from torchmetrics_amd.parallel import arena as _arena
from torchmetrics_amd.parallel.sync import distributed_available as _engine_dist_available
from torchmetrics_amd.parallel.sync import sync_state_dicts
from torchmetrics_amd.utilities.data import (
    _flatten,
    _squeeze_if_scalar,
    apply_to_collection,
    dim_zero_cat,
    dim_zero_max,
    dim_zero_mean,
    dim_zero_min,
    dim_zero_sum,
)
from torchmetrics_amd.utilities.exceptions import TorchMetricsUserError
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_single_or_multi_val
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils import profiling as _prof
from torchmetrics_amd.utils import validation as _validation

_REDUCTION_BY_NAME = {
    "sum": dim_zero_sum,
    "mean": dim_zero_mean,
    "max": dim_zero_max,
    "min": dim_zero_min,
    "cat": dim_zero_cat,
}

# reductions the engine all-reduces (everything else that is a tensor state is gathered)
_ENGINE_REDUCE_FNS = (dim_zero_sum, dim_zero_mean, dim_zero_max, dim_zero_min)

_NULL_CTX = nullcontext()

_CONST_ATTRS = (
    "higher_is_better",
    "is_differentiable",
    "full_state_update",
    "plot_lower_bound",
    "plot_upper_bound",
    "plot_legend_name",
)


def jit_distributed_available() -> bool:
    """True when ``torch.distributed`` is available and a default process group exists."""
    return _engine_dist_available()


_DESCRIPTORS: Dict[type, frozenset] = {}
_NO_NAMES: frozenset = frozenset()
# nn.Module lifecycle attributes that are not metric configuration (no fused-plan invalidation)
_LIFECYCLE_ATTRS = frozenset({"training", "call_super_init", "dump_patches"})


def _data_descriptors(cls: type) -> frozenset:
    """Names of the class-level data descriptors (properties with setters ...) of ``cls``; cached per class."""
    got = _DESCRIPTORS.get(cls)
    if got is None:
        names = set()
        for klass in cls.__mro__:
            for k, v in vars(klass).items():
                if hasattr(type(v), "__set__") or hasattr(type(v), "__delete__"):
                    names.add(k)
        got = _DESCRIPTORS[cls] = frozenset(names)
    return got


def _is_partial_view(t: Any) -> bool:
    """A strided tensor that covers only part of its storage (a view of a packed or cat arena)."""
    return (isinstance(t, Tensor) and t.layout == torch.strided
            and t.untyped_storage().nbytes() > t.numel() * t.element_size())


class _ChunkSnapshot:
    """A chunked list state's (materialised samples, pending chunks) entry held in the sync cache unbuilt."""

    __slots__ = ("entry",)

    def __init__(self, entry: Tuple[List[Tensor], List[Tuple[Tensor, List[int]]]]) -> None:
        self.entry = entry


def _interleave_gathered(flat: Tensor, sizes: Tensor, counts: Tensor) -> Tuple[Tensor, List[int]]:
    """Every rank's flat buffer / sample sizes / sample count, concatenated rank after rank by the engine -> the
    element-major sample order of the reference's per-element gather (sample 0 of every rank, then sample 1, ...;
    ``S/metric.py:442-457`` ``_flatten``), as ONE row gather of the flat buffer."""
    meta = torch.cat([counts.reshape(-1), sizes.reshape(-1)]).tolist()  # one host read of the metadata
    world = counts.numel()
    cnt, sz = meta[:world], meta[world:]
    rank_first = [0] * world
    for r in range(1, world):
        rank_first[r] = rank_first[r - 1] + cnt[r - 1]
    order = [rank_first[r] + e for e in range(max(cnt) if cnt else 0) for r in range(world) if e < cnt[r]]
    if order == list(range(len(sz))):
        return flat, sz
    row_start = [0] * len(sz)
    for i in range(1, len(sz)):
        row_start[i] = row_start[i - 1] + sz[i - 1]
    new_sizes = [sz[i] for i in order]
    lens = torch.tensor(new_sizes, dtype=torch.int64)
    starts = torch.tensor([row_start[i] for i in order], dtype=torch.int64)
    out_start = torch.cumsum(lens, 0) - lens
    idx = torch.repeat_interleave(starts - out_start, lens) + torch.arange(int(lens.sum()), dtype=torch.int64)
    return flat.index_select(0, idx.to(flat.device)), new_sizes


class Metric(Module, ABC):
    """Base class for all metrics.

    Subclasses register states with :meth:`add_state` and implement ``update`` and ``compute``.

    Keyword Args:
        compute_on_cpu: move list states to CPU after each ``update``.
        dist_sync_on_step: synchronise states inside ``forward`` (so the batch value is global).
        process_group: process group to sync over (default WORLD).
        dist_sync_fn: custom per-tensor gather; ``None`` selects the bucketed RCCL engine.
        distributed_available_fn: callable deciding whether we run distributed.
        sync_on_compute: synchronise states in ``compute``.
        compute_with_cache: cache the ``compute`` result until the next ``update``/``reset``.
    """

    __jit_ignored_attributes__ = ("device",)
    __jit_unused_properties__ = (
        "is_differentiable",
        "higher_is_better",
        "plot_lower_bound",
        "plot_upper_bound",
        "plot_legend_name",
        "metric_state",
        "_update_called",
    )
    is_differentiable: Optional[bool] = None
    higher_is_better: Optional[bool] = None
    full_state_update: Optional[bool] = None
    plot_lower_bound: Optional[float] = None
    plot_upper_bound: Optional[float] = None
    plot_legend_name: Optional[str] = None
    # fold `cat` list states into one tensor before compute() (see _consolidate_cat_lists); opt-out per class
    _fold_cat_lists: bool = True
    # forward(): fold the batch into unobserved SUM tensor states in place (see _merge_sums_in_place)
    _inplace_forward_merge: bool = True

    def __init__(self, **kwargs: Any) -> None:
        super().__init__()
        torch._C._log_api_usage_once(f"torchmetrics_amd.metric.{self.__class__.__name__}")
        self._device = torch.device("cpu")
        self._dtype = torch.get_default_dtype()

        def _bool_kw(name: str, default: bool) -> bool:
            val = kwargs.pop(name, default)
            if not isinstance(val, bool):
                raise ValueError(f"Expected keyword argument `{name}` to be an `bool` but got {val}")
            return val

        self.compute_on_cpu = _bool_kw("compute_on_cpu", False)
        self.dist_sync_on_step = _bool_kw("dist_sync_on_step", False)
        self.process_group = kwargs.pop("process_group", None)
        self.dist_sync_fn = kwargs.pop("dist_sync_fn", None)
        if self.dist_sync_fn is not None and not callable(self.dist_sync_fn):
            raise ValueError(
                f"Expected keyword argument `dist_sync_fn` to be an callable function but got {self.dist_sync_fn}"
            )
        self.distributed_available_fn = kwargs.pop("distributed_available_fn", None) or jit_distributed_available
        self.sync_on_compute = _bool_kw("sync_on_compute", True)
        self.compute_with_cache = _bool_kw("compute_with_cache", True)
        if kwargs:
            raise ValueError(f"Unexpected keyword arguments: {', '.join(f'`{a}`' for a in sorted(kwargs))}")

        self._update_signature = inspect.signature(self.update)
        self.update: Callable = self._wrap_update(self.update)  # type: ignore[method-assign]
        self.compute: Callable = self._wrap_compute(self.compute)  # type: ignore[method-assign]
        self._computed = None
        self._forward_cache = None
        self._update_count = 0
        self._to_sync = self.sync_on_compute
        self._should_unsync = True
        self._enable_grad = False
        self._dtype_convert = False

        self._defaults: Dict[str, Union[List, Tensor]] = {}
        self._persistent: Dict[str, bool] = {}
        self._reductions: Dict[str, Union[str, Callable[..., Any], None]] = {}

        self._is_synced = False
        self._cache: Optional[Dict[str, Union[List[Tensor], Tensor]]] = None
        # device-side validation flags (lazily allocated on first GPU update; see utils/validation.py)
        self._device_errors: Optional[Tensor] = None

    # ------------------------------------------------------------------------------------------------ properties
    @property
    def _update_called(self) -> bool:
        rank_zero_warn(
            "This property will be removed in 2.0.0. Use `Metric.updated_called` instead.",
            DeprecationWarning,
            stacklevel=2,
        )
        return self.update_called

    @property
    def update_called(self) -> bool:
        """``True`` if ``update``/``forward`` ran since construction or the last ``reset``."""
        return self._update_count > 0

    @property
    def update_count(self) -> int:
        return self._update_count

    @property
    def metric_state(self) -> Dict[str, Union[List[Tensor], Tensor]]:
        return {attr: getattr(self, attr) for attr in self._defaults}

    # ---------------------------------------------------------------------------------------------------- states
    def add_state(
        self,
        name: str,
        default: Union[list, Tensor],
        dist_reduce_fx: Optional[Union[str, Callable]] = None,
        persistent: bool = False,
    ) -> None:
        """Register a state: a tensor, or an empty list that ``update`` appends to.

        ``dist_reduce_fx`` in ``{"sum","mean","max","min","cat", None}`` or a callable applied to the rank-stacked
        state.
        """
        if not isinstance(default, (Tensor, list)) or (isinstance(default, list) and default):
            raise ValueError("state variable must be a tensor or any empty list (where you can append tensors)")
        if isinstance(dist_reduce_fx, str):
            if dist_reduce_fx not in _REDUCTION_BY_NAME:
                raise ValueError(
                    "`dist_reduce_fx` must be callable or one of ['mean', 'sum', 'cat', 'min', 'max', None]"
                )
            dist_reduce_fx = _REDUCTION_BY_NAME[dist_reduce_fx]
        elif dist_reduce_fx is not None and not callable(dist_reduce_fx):
            raise ValueError("`dist_reduce_fx` must be callable or one of ['mean', 'sum', 'cat', 'min', 'max', None]")
        if isinstance(default, Tensor):
            default = default.contiguous()
        setattr(self, name, default)
        self._defaults[name] = deepcopy(default)
        self.__dict__.pop("_default_packs", None)
        self._persistent[name] = persistent
        self._reductions[name] = dist_reduce_fx
        self._pack_states()

    def _pack_states(self) -> None:
        """Lay the reducible tensor states out as views of one buffer per (reduction, dtype, device)
        (:mod:`torchmetrics_amd.parallel.arena`); the sync engine then sends each bucket as one span."""
        _arena.pack([self], force=True)
        self.__dict__.pop("_arena_repacks", None)

    # ---------------------------------------------------------------------------------------------------- forward
    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        """Update the global state with the batch and return the metric value on the batch alone."""
        if self._is_synced:
            raise TorchMetricsUserError(
                "The Metric shouldn't be synced when performing ``forward``. "
                "HINT: Did you forget to call ``unsync`` ?."
            )
        if _prof.ENABLED:
            with _prof.range(f"tm.forward/{type(self).__name__}"):
                return self._forward_dispatch(*args, **kwargs)
        return self._forward_dispatch(*args, **kwargs)

    def _forward_dispatch(self, *args: Any, **kwargs: Any) -> Any:
        if self.full_state_update or self.full_state_update is None or self.dist_sync_on_step:
            self._forward_cache = self._forward_full_state_update(*args, **kwargs)
        else:
            self._forward_cache = self._forward_reduce_state_update(*args, **kwargs)
        return self._forward_cache

    def _enter_batch_mode(self) -> bool:
        self._to_sync = self.dist_sync_on_step
        self._should_unsync = False
        saved = self.compute_on_cpu
        self.__dict__["compute_on_cpu"] = False  # (lifecycle toggle: not a configuration change, see __setattr__)
        self._enable_grad = True
        return saved

    def _exit_batch_mode(self, saved_compute_on_cpu: bool) -> None:
        self._is_synced = False
        self._should_unsync = True
        self._to_sync = self.sync_on_compute
        self._computed = None
        self._enable_grad = False
        self.__dict__["compute_on_cpu"] = saved_compute_on_cpu
        if self.compute_on_cpu:
            self._move_list_states_to_cpu()

    def _batch_reset(self, separate: bool = False) -> None:
        """``reset()`` inside ``forward``: fresh default states for the batch (the saved global states are still
        referenced, so nothing can be refilled in place: every tensor state bucket is ONE clone of its packed
        defaults); the deferred-validation word and the global list arenas survive (they belong to the global
        state)."""
        d = self.__dict__
        if type(self).reset is not Metric.reset:
            # a subclass reset() may clear caches of its own: run it (keeping the global word and list arenas)
            d["_keep_device_errors"] = True
            try:
                self.reset()
            finally:
                d.pop("_keep_device_errors", None)
            return
        d.pop("_errors_checked_at", None)
        d["_update_count"] = 0
        d["_forward_cache"] = None
        d["_computed"] = None
        fresh: Dict[Tuple[Any, torch.dtype, torch.device], List[str]] = {}
        for attr, default in self._defaults.items():
            if isinstance(default, Tensor):
                cur = d.get(attr)
                dev = cur.device if isinstance(cur, Tensor) else default.device
                fresh.setdefault((_arena._reduce_kind(self._reductions[attr]), default.dtype, dev), []).append(attr)
            else:
                d[attr] = []
        self._fill_fresh(fresh, separate)
        d["_cache"] = None
        d["_is_synced"] = False

    def _restore_global(self, cache: Dict[str, Any], count: int, saved: bool) -> None:
        for attr, val in cache.items():
            setattr(self, attr, val)
        self._update_count = count
        self._exit_batch_mode(saved)

    def _forward_full_state_update(self, *args: Any, **kwargs: Any) -> Any:
        """Two ``update`` calls: one on the global state, one on a fresh state for the batch value."""
        self.update(*args, **kwargs)
        count = self._update_count
        saved = self._enter_batch_mode()
        cache = {attr: getattr(self, attr) for attr in self._defaults}
        grad_in = torch.is_grad_enabled() and any(
            isinstance(a, Tensor) and a.requires_grad for a in (*args, *kwargs.values()))
        try:
            self._batch_reset(separate=grad_in)
            self.update(*args, **kwargs)
            batch_val = self.compute()
        finally:
            # also on a raise (e.g. a validation bit surfacing in the batch compute): the global state and the
            # batch-mode flags come back exactly as they were
            self._restore_global(cache, count, saved)
        return batch_val

    def _forward_reduce_state_update(self, *args: Any, **kwargs: Any) -> Any:
        """One ``update`` on a fresh state, then fold the batch state into the saved global state."""
        global_state = {attr: getattr(self, attr) for attr in self._defaults}
        count = self._update_count
        saved = self._enter_batch_mode()
        # inputs carrying autograd history: the batch states must be separate leaves (in-place accumulation with
        # grad into views of one packed clone is refused by autograd)
        grad_in = torch.is_grad_enabled() and any(
            isinstance(a, Tensor) and a.requires_grad for a in (*args, *kwargs.values()))
        try:
            self._batch_reset(separate=grad_in)
            self.update(*args, **kwargs)
            batch_val = self.compute()
        except BaseException:
            self._restore_global(global_state, count, saved)
            raise
        self._update_count = count + 1
        with torch.no_grad():
            if self._inplace_forward_merge:
                self._merge_sums_in_place(global_state)
            self._reduce_states(global_state)
        self._exit_batch_mode(saved)
        return batch_val

    def _merge_sums_in_place(self, global_state: Dict[str, Any]) -> None:
        """forward()'s fold of the batch state into the global one, in place for SUM tensor states nothing else can
        observe: ``glob += batch`` on the global tensor (it stays in its packed arena, no new allocation) instead of
        ``glob + batch`` into a fresh tensor.  Nothing else may hold the global tensor -- only ``global_state`` and the
        locals below reference it (a returned ``compute()`` result aliasing it, a compute-group sibling or a user handle
        keeps the out-of-place merge, which the reference always does: S/metric.py:329-352).  Merged entries are
        handed to :meth:`_reduce_states` as already reduced."""
        pairs: List[Tuple[str, Tensor, Tensor]] = []
        # storage -> the global state's own tensors on it (the states and their packed-arena base); any other tensor
        # on that storage (a user view, a view returned by compute()) shows up in the storage's use count
        views: Dict[int, set] = {}
        for t in global_state.values():
            if isinstance(t, Tensor) and t.layout == torch.strided:
                own = views.setdefault(t.untyped_storage().data_ptr(), set())
                own.add(id(t))
                if t._base is not None:
                    own.add(id(t._base))
        t = own = None
        for attr in list(global_state):
            if self._reductions[attr] is not dim_zero_sum:
                continue
            # nothing but global_state may hold the global tensor object (a returned compute() result, a compute-group
            # sibling or a user handle keeps the out-of-place merge); asked before `glob` binds it to a local
            sole = _ops.sole_ref(global_state, attr)
            glob = global_state[attr]
            local = getattr(self, attr)
            if (not isinstance(glob, Tensor) or not isinstance(local, Tensor) or glob.requires_grad
                    or local.requires_grad or glob.layout != torch.strided or glob.shape != local.shape
                    or glob.dtype != torch.promote_types(glob.dtype, local.dtype) or glob.device != local.device):
                continue
            # the storage use count catches views of it (+1: the temporary storage handle)
            if not sole:
                continue
            stor = glob.untyped_storage()
            if torch._C._storage_Use_Count(stor._cdata) > 1 + len(views.get(stor.data_ptr(), ())):
                continue
            stor = None
            pairs.append((attr, glob, local))
        glob = local = stor = None
        if not pairs:
            return
        gspan = _arena.contiguous_span([g for _, g, _ in pairs]) if len(pairs) > 1 else None
        lspan = _arena.contiguous_span([t for _, _, t in pairs]) if gspan is not None else None
        if gspan is not None and lspan is not None and lspan.dtype == gspan.dtype:
            gspan.add_(lspan)  # the whole SUM bucket in one launch (both sides are packed spans in the same order)
        else:
            for _, g, t in pairs:
                g.add_(t)
        d = self.__dict__
        for attr, g, _ in pairs:
            d[attr] = g
            global_state[attr] = None  # consumed: _reduce_states skips it

    def _reduce_states(self, incoming_state: Dict[str, Any], only: Optional[str] = None) -> None:
        """Merge ``incoming_state`` (the pre-batch global state) with the current (batch) state (every state, or just
        ``only``)."""
        for attr in (self._defaults if only is None else (only,)):
            local = getattr(self, attr)
            glob = incoming_state[attr]
            if glob is None and attr in incoming_state:
                continue  # merged in place already (_merge_sums_in_place)
            fn = self._reductions[attr]
            if fn is dim_zero_sum:
                merged = glob + local
            elif fn is dim_zero_mean:
                merged = ((self._update_count - 1) * glob + local).float() / self._update_count
            elif fn is dim_zero_max:
                merged = torch.max(glob, local)
            elif fn is dim_zero_min:
                merged = torch.min(glob, local)
            elif fn is dim_zero_cat:
                merged = torch.cat([glob, local]) if isinstance(glob, Tensor) else glob + local
            elif fn is None and isinstance(glob, Tensor):
                merged = torch.stack([glob, local])
            elif fn is None and isinstance(glob, list):
                merged = _flatten([glob, local])
            elif callable(fn):
                merged = fn(torch.stack([glob, local]))
            else:
                raise TypeError(f"Unsupported reduce_fn: {fn}")
            setattr(self, attr, merged)

    # ------------------------------------------------------------------------------------------------------- sync
    def _static_gather_spec(self) -> Dict[str, Tuple[Tuple[int, ...], torch.dtype, Tuple[str, str]]]:
        """``{state: (configured shape, dtype, ident)}`` of the tensor states with a ``None`` / callable reduction:
        their ``add_state`` default fixes their shape on every rank, so the engine gathers them without the shape
        header (``parallel/sync.py`` static gather; a state that left that shape is caught by a signature)."""
        d = self.__dict__
        cached = d.get("_static_spec")
        if cached is not None and cached[0] == len(self._defaults):
            return cached[1]
        spec = {}
        for attr, default in self._defaults.items():
            fn = self._reductions.get(attr)
            if isinstance(default, Tensor) and fn is not dim_zero_cat and (
                    fn is None or (callable(fn) and fn not in _ENGINE_REDUCE_FNS)):
                spec[attr] = (tuple(default.shape), default.dtype, (type(self).__qualname__, attr))
        d["_static_spec"] = (len(self._defaults), spec)
        return spec

    def _compute_sync_override(self) -> Optional[Tuple[Dict[str, Tensor], Dict[str, Callable]]]:
        """States to sync INSTEAD of the metric's own when the sync only serves this ``compute()`` (``None``: the
        states themselves).  A metric whose compute needs less than its states (calibration error: its bins, not the
        sample lists) overrides this and :meth:`_compute_sync_finish`; ``sync()`` / ``sync_context`` always sync the
        real states (reference contract, ``S/metric.py:427-457``)."""
        return None

    def _compute_sync_finish(self, synced: Dict[str, Any]) -> None:
        """Receives the synced override states of :meth:`_compute_sync_override` (this metric and every member of
        its compute group)."""

    def _sync_dist(self, dist_sync_fn: Optional[Callable] = None, process_group: Optional[Any] = None) -> None:
        group = process_group or self.process_group
        if dist_sync_fn is None and self.__dict__.get("_in_compute"):
            override = self._compute_sync_override()
            if override is not None:
                dev = next((v.device for v in override[0].values() if isinstance(v, Tensor) and v.is_cuda), None)
                err = self._device_error_buffer(dev) if dev is not None else None
                synced = sync_state_dicts([override], group=group, err_word=err, narrow_word=err)[0]
                self._compute_sync_finish(synced)
                if err is not None:
                    self.__dict__["_sync_word_pending"] = True
                return
        packed = self._packed_sync_plan(group) if dist_sync_fn is None and self._packed_sync_states else {}
        states = {attr: getattr(self, attr) for attr in self._reductions if attr not in packed}
        if dist_sync_fn is None:
            reductions = self._reductions
            if packed:
                # a chunked list state crosses as its flat buffer + sample sizes (two cat items of the same engine
                # call) instead of one list element per sample; re-interleaved element-major afterwards
                reductions = {a: f for a, f in self._reductions.items() if a not in packed}
                for attr, (flat, sizes) in packed.items():
                    dev = flat.device if flat is not None else self.device
                    states[attr + "\0flat"] = [flat] if flat is not None else []
                    states[attr + "\0sizes"] = [torch.tensor(sizes, dtype=torch.int64, device=dev)] if sizes else []
                    states[attr + "\0n"] = [torch.tensor([len(sizes)], dtype=torch.int64, device=dev)]
                    for k in ("\0flat", "\0sizes", "\0n"):
                        reductions[attr + k] = dim_zero_cat
            # (sync() packed the reducible states into their arena before caching them: each bucket is one span)
            # a one-shot xGMI bucket reports failure in this metric's validation word: compute() reads the word after
            # the sync (sync() reads it right away when called on its own)
            dev = next((v.device for v in states.values() if isinstance(v, Tensor) and v.is_cuda), None)
            err = self._device_error_buffer(dev) if dev is not None else None
            # inside compute() a narrow-wire overflow is reported in the same word (no host read in the sync)
            narrow = err if self.__dict__.get("_defer_narrow") else None
            synced = sync_state_dicts([(states, reductions, self._static_gather_spec())], group=group, err_word=err,
                                      narrow_word=narrow)[0]
            for attr in packed:
                flat, sizes, n = synced.pop(attr + "\0flat"), synced.pop(attr + "\0sizes"), synced.pop(attr + "\0n")
                setattr(self, attr, [])
                if isinstance(flat, Tensor) and isinstance(sizes, Tensor) and sizes.numel():
                    flat, order = _interleave_gathered(flat, sizes, n)
                    self._append_chunk(attr, flat, order)
            for attr, val in synced.items():
                setattr(self, attr, val)
            if err is not None:
                self.__dict__["_sync_word_pending"] = True
            return
        # user-supplied per-tensor gather: reference contract, one call per state tensor
        for attr, fn in self._reductions.items():
            if fn is dim_zero_cat and isinstance(states[attr], list) and len(states[attr]) > 1:
                states[attr] = [dim_zero_cat(states[attr])]
        gathered = apply_to_collection(states, Tensor, dist_sync_fn, group=group)
        for attr, fn in self._reductions.items():
            val = gathered[attr]
            if isinstance(val, list) and len(val) == 0:
                setattr(self, attr, [])
                continue
            if isinstance(val[0], Tensor):
                val = torch.stack(val)
            elif isinstance(val[0], list):
                val = _flatten(val)
            if not (callable(fn) or fn is None):
                raise TypeError("reduction_fn must be callable or None")
            setattr(self, attr, fn(val) if fn is not None else val)

    def _wrap_update(self, update: Callable) -> Callable:
        # Host cost matters here: an MI355X update kernel runs in a few us, so this wrapper writes its bookkeeping
        # straight into __dict__ (nn.Module.__setattr__ costs ~1 us per call) and flips grad mode with the raw C
        # toggle instead of a context-manager object.
        state = self.__dict__
        set_grad = torch._C._set_grad_enabled

        @functools.wraps(update)
        def wrapped_func(*args: Any, **kwargs: Any) -> None:
            if _prof.ENABLED:
                _prof.push(f"tm.update/{type(self).__name__}")
                try:
                    return _update_body(*args, **kwargs)
                finally:
                    _prof.pop()
            return _update_body(*args, **kwargs)

        def _update_body(*args: Any, **kwargs: Any) -> None:
            state["_computed"] = None
            state["_update_count"] += 1
            prev = torch.is_grad_enabled()
            want = state["_enable_grad"]
            if prev != want:
                set_grad(want)
            try:
                update(*args, **kwargs)
            except RuntimeError as err:
                if "Expected all tensors to be on" in str(err):
                    raise RuntimeError(
                        "Encountered different devices in metric calculation (see stacktrace for details)."
                        " This could be due to the metric class not being on the same device as input."
                        f" Instead of `metric={self.__class__.__name__}(...)` try to do"
                        f" `metric={self.__class__.__name__}(...).to(device)` where"
                        " device corresponds to the device of the input."
                    ) from err
                raise err
            finally:
                if prev != want:
                    set_grad(prev)
            if _validation.STRICT and state["_device_errors"] is not None:
                self._raise_device_errors()
            if self.compute_on_cpu:
                self._move_list_states_to_cpu()

        return wrapped_func

    def _device_error_buffer(self, device: torch.device) -> Tensor:
        """Per-metric int32 flag word the HIP kernels ``atomicOr`` validation failures into."""
        buf = self._device_errors
        if buf is None or buf.device != device:
            buf = torch.zeros(1, dtype=torch.int32, device=device)
            self._device_errors = buf
        return buf

    def _raise_device_errors(self, only: int = 0) -> None:
        """Read the deferred-validation word (one device sync) and raise what it holds; ``only``: a bit mask -- raise
        just those bits and leave the others for ``compute()``."""
        buf = self._device_errors
        self.__dict__.pop("_sync_word_pending", None)
        if buf is None:
            return
        code = _ops.read_word(buf)
        if code & _validation.NARROW_RETRY and not only:
            code = self._narrow_resync(buf, code)
        if only:
            code &= only
        if code:
            if only:
                buf.bitwise_and_(~only)
            else:
                buf.zero_()
            _validation.raise_for_code(code, self)

    def _narrow_resync(self, buf: Tensor, code: int) -> int:
        """A narrow-wire bucket of compute()'s sync overflowed (``NARROW_RETRY``; every rank sees the same summed
        check slots, so every rank is here): move those buckets one width up and sync again, checking the wire inline
        this time.  Runs before any other bit of the word raises, so no rank leaves a peer inside the re-sync."""
        from torchmetrics_amd.parallel.sync import narrow_resolve

        while code & _validation.NARROW_RETRY:
            buf.bitwise_and_(~_validation.NARROW_RETRY)
            narrow_resolve(buf)
            if self._is_synced:
                self.unsync()
                self.sync(dist_sync_fn=self.dist_sync_fn)
            code = int(buf.item())
        return code

    def _move_list_states_to_cpu(self) -> None:
        for key in self._defaults:
            val = getattr(self, key)
            if isinstance(val, Sequence):
                setattr(self, key, [v.to("cpu") for v in val])

    def sync(
        self,
        dist_sync_fn: Optional[Callable] = None,
        process_group: Optional[Any] = None,
        should_sync: bool = True,
        distributed_available: Optional[Callable] = None,
    ) -> None:
        """Synchronise states across processes (no-op when not distributed or ``should_sync=False``)."""
        if self._is_synced and should_sync:
            raise TorchMetricsUserError("The Metric has already been synced.")
        if distributed_available is None and self.distributed_available_fn is not None:
            distributed_available = self.distributed_available_fn
        is_distributed = distributed_available() if callable(distributed_available) else None
        if not should_sync or not is_distributed:
            return
        if dist_sync_fn is None and self.dist_sync_fn is None:
            _arena.pack([self])  # no-op when laid out already; BEFORE the cache, so unsync restores the packed views
        chunks = self.__dict__.get("_chunks")
        self._cache = {attr: (_ChunkSnapshot(chunks[attr]) if chunks and attr in chunks else getattr(self, attr))
                       for attr in self._defaults}
        self._sync_dist(dist_sync_fn, process_group=process_group)
        self._is_synced = True
        if self.__dict__.get("_sync_word_pending") and not self.__dict__.get("_in_compute"):
            # stand-alone sync(): a failed one-shot bucket must raise now, before anyone reads the states
            try:
                self._raise_device_errors(only=_validation.ONESHOT_FAILED)
            except RuntimeError:
                self.unsync()
                raise

    def unsync(self, should_unsync: bool = True) -> None:
        """Restore the local (pre-sync) states."""
        if not should_unsync:
            return
        if not self._is_synced:
            raise TorchMetricsUserError("The Metric has already been un-synced.")
        if self._cache is None:
            raise TorchMetricsUserError("The internal cache should exist to unsync the Metric.")
        for attr, val in self._cache.items():
            if isinstance(val, _ChunkSnapshot):  # a chunked list state goes back to its chunks, still unbuilt
                setattr(self, attr, [])
                d = self.__dict__
                del d[attr]
                d.setdefault("_chunks", {})[attr] = val.entry
            else:
                setattr(self, attr, val)
        self._is_synced = False
        self._cache = None

    @contextmanager
    def sync_context(
        self,
        dist_sync_fn: Optional[Callable] = None,
        process_group: Optional[Any] = None,
        should_sync: bool = True,
        should_unsync: bool = True,
        distributed_available: Optional[Callable] = None,
    ) -> Generator:
        """Sync on entry, restore local states on exit."""
        self.sync(
            dist_sync_fn=dist_sync_fn,
            process_group=process_group,
            should_sync=should_sync,
            distributed_available=distributed_available,
        )
        yield
        self.unsync(should_unsync=self._is_synced and should_unsync)

    def _wrap_compute(self, compute: Callable) -> Callable:
        @functools.wraps(compute)
        def wrapped_func(*args: Any, **kwargs: Any) -> Any:
            if _prof.ENABLED:
                _prof.push(f"tm.compute/{type(self).__name__}")
                try:
                    return _compute_body(*args, **kwargs)
                finally:
                    _prof.pop()
            return _compute_body(*args, **kwargs)

        def _compute_body(*args: Any, **kwargs: Any) -> Any:
            if not self.update_called:
                rank_zero_warn(
                    f"The ``compute`` method of metric {self.__class__.__name__}"
                    " was called before the ``update`` method which may lead to errors,"
                    " as metric states have not yet been updated.",
                    UserWarning,
                )
            state = self.__dict__
            if state["_computed"] is not None:
                return state["_computed"]
            if self._fold_cat_lists:
                self._consolidate_cat_lists()
            avail = state["distributed_available_fn"]
            if not state["_is_synced"] and not (state["_to_sync"] and callable(avail) and avail()):
                # nothing to gather: skip the sync / unsync bookkeeping (attribute traffic per call)
                self._check_errors_once(state)
                value = compute(*args, **kwargs)
                value = (value.squeeze() if value.numel() == 1 else value) if isinstance(value, Tensor) \
                    else _squeeze_if_scalar(value)
            else:
                # sync FIRST, then read the validation word once: every rank has finished its collectives before any
                # rank raises (a rank raising before the sync would leave its peers waiting), and the same read
                # covers a failed one-shot bucket of this very sync
                state["_in_compute"] = state["_defer_narrow"] = True
                try:
                    self.sync(dist_sync_fn=self.dist_sync_fn, should_sync=self._to_sync)
                finally:
                    state.pop("_in_compute", None)
                    state.pop("_defer_narrow", None)
                try:
                    self._check_errors_once(state)
                    value = _squeeze_if_scalar(compute(*args, **kwargs))
                finally:
                    # also on a raise: the local states come back, accumulation can go on
                    self.unsync(should_unsync=self._is_synced and self._should_unsync)
            if state["compute_with_cache"]:
                state["_computed"] = value
            return value

        return wrapped_func

    def _check_errors_once(self, state: Dict[str, Any]) -> None:
        """Raise what the deferred-validation word holds (one 4-byte device read).  The word only changes through
        update() / graph replays (which bump ``_update_count``) and through a sync's one-shot buckets: a word read
        clean at this count, with no sync since, is still clean (no device sync on repeated ``compute()`` calls)."""
        if state["_device_errors"] is None:
            return
        pending = state.get("_sync_word_pending", False)
        if state.pop("_device_errors_clean", False) and not pending:
            return
        if pending or state.get("_errors_checked_at") != state["_update_count"]:
            self._raise_device_errors()
            state["_errors_checked_at"] = state["_update_count"]

    _fold_every: int = 1  # cat-list batches pending before compute() folds them into the arena

    def _consolidate_cat_lists(self) -> None:
        """Replace the elements of every ``cat`` list state by their concatenation, in place (same list object).

        A list state grows by one tensor per update; ``compute()`` concatenates it.  Without this, a loop that calls
        ``compute()`` every step (per-step logging) re-concatenates every batch seen so far each time: O(steps)
        launches-worth of host work per call, O(steps^2) overall.  Folding the list into one tensor keeps each
        ``compute()`` at one ``cat`` of [accumulated, new batches].  The concatenated contents -- the only thing a
        ``cat`` reduction defines -- are unchanged (the reference folds cat lists the same way when it syncs them,
        ``S/metric.py:431-433``).  On by default; a class whose compute looks at the list's element structure opts out
        with ``_fold_cat_lists = False`` (EED averages per-update scores; ``None``-reduction lists such as mAP's
        per-image states are never folded)."""
        if not self._fold_cat_lists:
            return
        d = self.__dict__
        cats = d.get("_cat_attrs")
        if cats is None or cats[0] is not self._reductions or cats[1] != len(self._reductions):
            # the `cat` states, recomputed only when the reduction table changes (most metrics have none)
            cats = d["_cat_attrs"] = (self._reductions, len(self._reductions),
                                      tuple(a for a, fn in self._reductions.items() if fn is dim_zero_cat))
        for attr in cats[2]:
            val = d[attr] if attr in d else getattr(self, attr)
            # a class whose compute() usually does not read the list (the calibration error, served by its bin cache)
            # folds only once `_fold_every` batches are pending
            if isinstance(val, list) and len(val) > self._fold_every:
                val[:] = [self._fold_into_arena(attr, val)]

    def _fold_into_arena(self, attr: str, parts: List[Any]) -> Any:
        """Concatenate a ``cat`` list state into its growable HBM arena.

        The fold's result is a view ``buf[:rows]`` of a per-state buffer.  When the list is that view plus new
        batches, only the new batches are copied (one ``cat`` into ``buf[rows:]``); the buffer is re-allocated with
        amortised doubling when they do not fit, so per-step ``compute()`` costs O(new rows) instead of re-copying the
        whole history.  The first fold allocates exactly what it needs (a compute-once evaluation carries no slack).
        Autograd, mixed dtypes / devices / trailing shapes and ``forward()``'s batch states take a plain ``cat``."""
        d = self.__dict__
        if d.get("_enable_grad"):
            return dim_zero_cat(parts)  # forward()'s batch state: never touch the global state's arena
        first = parts[0]
        if not isinstance(first, Tensor) or first.ndim == 0:
            return dim_zero_cat(parts)
        tail, dtype, dev = first.shape[1:], first.dtype, first.device
        grad = torch.is_grad_enabled()
        for p in parts:
            if (not isinstance(p, Tensor) or p.ndim == 0 or p.shape[1:] != tail or p.dtype != dtype or p.device != dev
                    or p.layout != torch.strided or (grad and p.requires_grad)):
                return dim_zero_cat(parts)
        arenas = d.get("_cat_arenas")
        if arenas is None:
            arenas = d["_cat_arenas"] = {}
        entry = arenas.get(attr)
        if entry is not None and entry[1] is first and entry[0].dtype == dtype and entry[0].device == dev:
            buf, used, new = entry[0], first.shape[0], parts[1:]
        else:
            buf, used, new = None, 0, parts
        need = used + sum(p.shape[0] for p in new)
        if buf is None or need > buf.shape[0]:
            cap = need if buf is None else max(need, 2 * buf.shape[0])
            grown = torch.empty((cap,) + tuple(tail), dtype=dtype, device=dev)
            if used:
                grown[:used].copy_(buf[:used])
            buf = grown
        torch.cat(new, dim=0, out=buf[used:need])
        view = buf[:need]
        arenas[attr] = (buf, view)
        return view

    @abstractmethod
    def update(self, *_: Any, **__: Any) -> None:
        """Update the states with a batch."""

    @abstractmethod
    def compute(self) -> Any:
        """Compute the metric value from the (synced) states."""

    def plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        """Plot a single or multiple values from the metric (every reference subclass does exactly this)."""
        return self._plot(val, ax)

    def _plot(self, val: Any = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        val = val if val is not None else self.compute()
        return plot_single_or_multi_val(
            val,
            ax=ax,
            higher_is_better=self.higher_is_better,
            name=self.__class__.__name__,
            lower_bound=self.plot_lower_bound,
            upper_bound=self.plot_upper_bound,
            legend_name=self.plot_legend_name,
        )

    def reset(self) -> None:
        """Reset all states to their defaults.

        A public reset also clears the deferred-validation word (stream-ordered ``zero_``, no host sync): a bad batch
        that was never computed must not raise for data that is no longer in the state.
        """
        d = self.__dict__
        for name in d.pop("_chunks", None) or ():
            d[name] = []  # pending chunks of a list state: dropped with the state (rebuilt below)
        d.pop("_errors_checked_at", None)
        d.pop("_arena_repacks", None)  # a reset's fresh states are re-packed at the next sync without counting
        if not d.get("_keep_device_errors"):
            d.pop("_cat_arenas", None)  # (forward()'s batch reset keeps the global state's arenas)
        if not d.get("_keep_device_errors") and d.get("_device_errors") is not None:
            self._device_errors.zero_()
        self._update_count = 0
        self._forward_cache = None
        self._computed = None
        # storage -> this metric's own tensors on it: its states and their view bases (a packed arena's buffer)
        views: Dict[int, set] = {}
        for attr in self._defaults:
            t = d.get(attr)
            if isinstance(t, Tensor) and t.layout == torch.strided:
                own = views.setdefault(t.untyped_storage().data_ptr(), set())
                own.add(id(t))
                if t._base is not None:
                    own.add(id(t._base))
        t = own = None  # (the loop variables would count as references below)
        fresh: Dict[Tuple[Any, torch.dtype, torch.device], List[str]] = {}
        for attr, default in self._defaults.items():
            # nothing but the metric's __dict__ may hold the state object (asked before `cur` binds it)
            sole = isinstance(default, Tensor) and _ops.sole_ref(d, attr)
            cur = d[attr] if attr in d else getattr(self, attr)
            if isinstance(default, Tensor):
                allowed = 1 + len(views.get(cur.untyped_storage().data_ptr(), ())) if cur.layout == torch.strided else 2
                if not (sole and self._refill_in_place(cur, default, allowed)):
                    key = (_arena._reduce_kind(self._reductions[attr]), default.dtype, cur.device)
                    fresh.setdefault(key, []).append(attr)
            else:
                setattr(self, attr, [])
            del cur
        self._fill_fresh(fresh)
        self._cache = None
        self._is_synced = False

    def _fill_fresh(self, fresh: Dict[Tuple[Any, torch.dtype, torch.device], List[str]],
                    separate: bool = False) -> None:
        """Rebind ``fresh`` states (grouped by (reduction, dtype, device)) to copies of their defaults: several states of
        one bucket are views of ONE clone of their packed defaults -- already laid out as the sync engine's arena span."""
        for (kind, _dt, dev), attrs in fresh.items():
            if separate or kind is None or len(attrs) == 1:
                for attr in attrs:
                    setattr(self, attr, self._defaults[attr].detach().clone().to(dev))
            else:
                flat = self._packed_default(tuple(attrs), dev).clone()
                off = 0
                for attr in attrs:
                    dflt = self._defaults[attr]
                    n = dflt.numel()
                    setattr(self, attr, flat[off : off + n].view(dflt.shape))
                    off += n

    def _packed_default(self, attrs: Tuple[str, ...], device: torch.device) -> Tensor:
        """The defaults of ``attrs`` back to back on ``device`` (cached until the defaults change)."""
        cache = self.__dict__.get("_default_packs")
        if cache is None:
            cache = self.__dict__["_default_packs"] = {}
        key = (attrs, device)
        flat = cache.get(key)
        if flat is None:
            flat = torch.cat([self._defaults[a].detach().reshape(-1).to(device) for a in attrs])
            cache[key] = flat
        return flat

    @staticmethod
    def _refill_in_place(cur: Any, default: Tensor, allowed: int = 2) -> bool:
        """Reset a tensor state by refilling its own memory when nothing else can observe it (the caller checked that
        no other Python reference to the tensor exists (a returned ``compute()`` result, a forward()'s saved global state, a compute-group
        sibling, a user handle); here: no other tensor on its storage (views) but this metric's own states of the same
        packed arena (``allowed`` = 1 + their count).  Then the refill is invisible, and the
        state keeps its warm memory (allocator block, TLB and cache residency) -- the reference's reset always
        allocates a fresh clone of the default (S/metric.py:673-688), which is what happens here otherwise."""
        if not isinstance(cur, Tensor) or cur.requires_grad or cur.layout != torch.strided:
            return False
        if cur.shape != default.shape or cur.dtype != default.dtype or cur.device != default.device:
            return False
        if not cur.is_contiguous() or torch._C._storage_Use_Count(cur.untyped_storage()._cdata) > allowed:
            return False
        cur.copy_(default)
        return True

    def clone(self) -> "Metric":
        return deepcopy(self)

    # ------------------------------------------------------------------------------------------------- pickling
    def __getstate__(self) -> Dict[str, Any]:
        self._materialize_all_chunks()
        state = {k: v for k, v in self.__dict__.items()
                 if k not in ("update", "compute", "forward", "_update_signature", "_cat_arenas", "_default_packs",
                              "_cat_attrs")}
        for key in self._defaults:  # a folded list state: its own rows only, not the arena's spare capacity
            cur = state.get(key)
            if isinstance(cur, list) and any(_is_partial_view(v) for v in cur):
                state[key] = [v.clone() if _is_partial_view(v) else v for v in cur]
        return state

    def __setstate__(self, state: Dict[str, Any]) -> None:
        self.__dict__.update(state)
        self._update_signature = inspect.signature(self.update)
        self.update: Callable = self._wrap_update(self.update)  # type: ignore[method-assign]
        self.compute: Callable = self._wrap_compute(self.compute)  # type: ignore[method-assign]
        self._install_native_update()
        self._install_native_forward()

    # ------------------------------------------------------------------------------------- chunked list states
    def _append_chunk(self, name: str, flat: Tensor, sizes: List[int]) -> None:
        """Append ``len(sizes)`` per-sample tensors to list state ``name`` as ONE chunk: ``flat`` holds them back to
        back along dim 0 (``sizes[i]`` rows each).  A list update of a whole batch is then one ``cat`` instead of one
        Python append (and one tensor) per sample -- MeanAveragePrecision appends 9 per image.  The per-sample views
        are only built when something reads the state as a list (first attribute access: ``__getattr__``; state_dict,
        sync, pickling, ``metric_state``); computes that understand chunks read them flat (:meth:`_packed_state`)."""
        d = self.__dict__
        chunks = d.get("_chunks")
        if chunks is None:
            chunks = d["_chunks"] = {}
        entry = chunks.get(name)
        if entry is None:
            entry = chunks[name] = (d.pop(name), [])  # (the samples already materialised, pending chunks)
        entry[1].append((flat, list(sizes)))

    def __getattr__(self, name: str) -> Any:
        chunks = self.__dict__.get("_chunks")
        if chunks and name in chunks:
            return self._materialize_chunks(name)
        return super().__getattr__(name)

    # list states this class lets the sync engine move as ONE flat buffer + sample sizes (``_packed_state``) instead
    # of one list element per sample; the ranks agree on it per call (one flag all-reduce), since a rank whose samples
    # do not stack (ragged trailing shapes, mixed dtypes) must keep the element-wise form on every rank
    _packed_sync_states: Tuple[str, ...] = ()

    def _packed_sync_plan(self, group: Optional[Any]) -> Dict[str, Tuple[Optional[Tensor], List[int]]]:
        local: Dict[str, Tuple[Optional[Tensor], List[int]]] = {}
        ok = []
        for attr in self._packed_sync_states:
            flat, sizes = self._packed_state(attr)
            local[attr] = (flat, sizes)
            ok.append(1 if (flat is not None and flat.ndim >= 1) or not sizes else 0)
        dev = next((f.device for f, _ in local.values() if f is not None), self.device)
        from torchmetrics_amd.parallel.sync import _device_comm

        flag_dev = torch.device("cuda", torch.cuda.current_device()) if _device_comm(group) else torch.device("cpu")
        flags = torch.tensor(ok, dtype=torch.int32, device=flag_dev)
        torch.distributed.all_reduce(flags, op=torch.distributed.ReduceOp.MIN, group=group)
        del dev
        return {a: local[a] for a, f in zip(self._packed_sync_states, flags.tolist()) if f}

    def _materialize_chunks(self, name: str) -> List[Tensor]:
        base, pending = self.__dict__["_chunks"].pop(name)
        for flat, sizes in pending:
            base.extend(torch.split(flat, sizes))
        self.__dict__[name] = base
        return base

    def _materialize_all_chunks(self) -> None:
        chunks = self.__dict__.get("_chunks")
        for name in list(chunks or ()):
            self._materialize_chunks(name)

    def _packed_state(self, name: str) -> Tuple[Optional[Tensor], List[int]]:
        """List state ``name`` as ``(flat, sizes)`` -- the samples back to back along dim 0 (one ``cat`` of the pending
        chunks) and each sample's row count -- without building per-sample views.  ``(None, sizes)`` when the samples
        do not stack that way (a ragged trailing shape, several devices / dtypes): read the list then."""
        d = self.__dict__
        chunks = d.get("_chunks")
        if chunks and name in chunks:
            base, pending = chunks[name]
            parts = list(base) + [f for f, _ in pending]
            sizes = [x.shape[0] if x.ndim else 1 for x in base] + [n for _, ns in pending for n in ns]
        else:
            parts = d[name] if name in d else getattr(self, name)
            sizes = [x.shape[0] if x.ndim else 1 for x in parts]
        if not parts:
            return None, sizes
        tail = parts[0].shape[1:]
        if any(p.ndim == 0 or p.shape[1:] != tail or p.dtype != parts[0].dtype or p.device != parts[0].device
               for p in parts):
            return None, sizes
        return (parts[0] if len(parts) == 1 else torch.cat(parts)), sizes

    def __prepare_scriptable__(self) -> "Metric":
        """``torch.jit.script`` compiles the class's methods; the native C++ entry points installed as instance
        attributes (``csrc/bindings/fastcall.cpp`` NativeUpdate / NativeForward) are not Python functions, so the
        module handed to the compiler is a shallow COPY without them (its Python ``update`` / ``forward`` take over:
        same results, the same state tensors).  The eager metric itself keeps its native entry points: scripting it
        once does not take the fast path away for the rest of the run.  The copy gets its own ``_modules`` dict, which
        the compiler's recursion may rewrite."""
        clone = object.__new__(type(self))
        d = clone.__dict__
        d.update(self.__dict__)
        d["_modules"] = type(self._modules)(self._modules)
        if type(d.get("forward")).__name__ == "NativeForward":
            del d["forward"]
        if type(d.get("update")).__name__ == "NativeUpdate":
            d["update"] = d["update"].fallback
        d.pop("_default_packs", None)  # a cache keyed by (names, device) tuples, which TorchScript cannot type
        return clone

    def _install_native_update(self) -> None:
        """Hook: classes with a native ``update`` entry point install it over the Python wrapper here."""

    def _install_native_forward(self) -> None:
        """Hook: classes with a native ``forward`` (``csrc/bindings/fastcall.cpp`` ``NativeForward``) install it as the
        instance's ``forward`` here (calls off its fast path run :meth:`Metric.forward`)."""

    def __setattr__(self, name: str, value: Any) -> None:
        if name in _CONST_ATTRS:
            raise RuntimeError(f"Can't change const `{name}`.")
        d = self.__dict__
        chunks = d.get("_chunks")
        if chunks and name in chunks:
            del chunks[name]  # the state is rebound (reset, sync, load): its pending chunks are no longer its value
        if (name[0] != "_" and name not in _LIFECYCLE_ATTRS and name not in d.get("_defaults", _NO_NAMES)
                and not (name in d and d[name] is value and isinstance(value, (str, int, float, bool, type(None))))):
            # a configuration attribute (average, num_classes, ...) that changes: plans recorded from this metric
            # (utils/fused_compute.py) check the version before replaying.  nn.Module's own mode flag (``training``,
            # set on every member by train() / eval()) is not configuration: a train / validate loop must not
            # invalidate the plan at each mode switch
            d["_cfg_version"] = d.get("_cfg_version", 0) + 1
        # fast path for the bookkeeping attributes and states the lifecycle rebinds on every update / compute /
        # forward (nn.Module.__setattr__ costs ~1.5-2.5 us per call): an attribute this instance already holds as a
        # plain value, that is no parameter, buffer, sub-module or class-level data descriptor, is rebound in place
        if (name in d and not isinstance(value, (Parameter, Module)) and name not in d.get("_parameters", _NO_NAMES)
                and name not in d.get("_buffers", _NO_NAMES) and name not in d.get("_modules", _NO_NAMES)
                and name not in _data_descriptors(type(self))):
            d[name] = value
            return
        super().__setattr__(name, value)

    # ------------------------------------------------------------------------------------------ device / dtype
    @property
    def device(self) -> "torch.device":
        return self._device

    @property
    def dtype(self) -> "torch.dtype":
        return self._dtype

    def type(self, dst_type: Union[str, torch.dtype]) -> "Metric":  # noqa: A003
        """No-op; use :meth:`set_dtype` (metric states keep their dtype under ``.half()`` etc.)."""
        return self

    def float(self) -> "Metric":  # noqa: A003
        return self

    def double(self) -> "Metric":
        return self

    def half(self) -> "Metric":
        return self

    def set_dtype(self, dst_type: Union[str, torch.dtype]) -> "Metric":
        """Convert floating states to ``dst_type``."""
        self._dtype_convert = True
        out = super().type(dst_type)
        out._dtype_convert = False
        return out

    def _apply(self, fn: Callable, exclude_state: Sequence[str] = "") -> Module:  # type: ignore[override]
        this = super()._apply(fn)
        fs = str(fn)
        is_dtype_cast = any(f in fs for f in ("Module.type", "Module.half", "Module.float", "Module.double", "Module.bfloat16"))
        if not self._dtype_convert and is_dtype_cast:
            return this
        for key, value in this._defaults.items():
            if key in exclude_state:
                continue
            if isinstance(value, Tensor):
                this._defaults[key] = fn(value)
            elif isinstance(value, Sequence):
                this._defaults[key] = [fn(v) for v in value]
            cur = getattr(this, key)
            if isinstance(cur, Tensor):
                setattr(this, key, fn(cur))
            elif isinstance(cur, Sequence):
                setattr(this, key, [fn(v) for v in cur])
            else:
                raise TypeError(
                    f"Expected metric state to be either a Tensor or a list of Tensor, but encountered {cur}"
                )
        this.__dict__["_cfg_version"] = this.__dict__.get("_cfg_version", 0) + 1  # device / dtype moved
        this.__dict__.pop("_cat_arenas", None)  # folded list states were moved out of their arenas
        this.__dict__.pop("_default_packs", None)  # the defaults were moved / cast
        this._pack_states()  # the moved / cast states are separate tensors again: one buffer per bucket
        probe = fn(torch.zeros(1, device=self.device))
        self._device = probe.device
        self._dtype = probe.dtype
        if this._computed is not None:
            this._computed = apply_to_collection(this._computed, Tensor, fn)
        if this._forward_cache is not None:
            this._forward_cache = apply_to_collection(this._forward_cache, Tensor, fn)
        if this._device_errors is not None and this._device_errors.device != self._device:
            this._device_errors = None
        return this

    # ------------------------------------------------------------------------------------------- checkpointing
    def persistent(self, mode: bool = False) -> None:
        for key in self._persistent:
            self._persistent[key] = mode

    def state_dict(  # type: ignore[override]
        self,
        destination: Optional[Dict[str, Any]] = None,
        prefix: str = "",
        keep_vars: bool = False,
    ) -> Dict[str, Any]:
        destination = super().state_dict(destination=destination, prefix=prefix, keep_vars=keep_vars)  # type: ignore
        for key in self._defaults:
            if not self._persistent[key]:
                continue
            cur = getattr(self, key)
            if not keep_vars:
                if isinstance(cur, Tensor):
                    cur = cur.detach()
                elif isinstance(cur, list):
                    cur = [v.detach() if isinstance(v, Tensor) else v for v in cur]
            if _is_partial_view(cur):
                # a view of the packed arena: copy just its own elements (deepcopy would copy the whole buffer)
                cur = cur.detach().clone().requires_grad_(cur.requires_grad)
            elif isinstance(cur, list) and any(_is_partial_view(v) for v in cur):
                cur = [v.detach().clone() if _is_partial_view(v) else deepcopy(v) for v in cur]  # folded cat arena
            else:
                cur = deepcopy(cur)
            destination[prefix + key] = cur
        return destination

    def _load_from_state_dict(
        self,
        state_dict: dict,
        prefix: str,
        local_metadata: dict,
        strict: bool,
        missing_keys: List[str],
        unexpected_keys: List[str],
        error_msgs: List[str],
    ) -> None:
        for key in self._defaults:
            name = prefix + key
            if name in state_dict:
                setattr(self, key, state_dict.pop(name))
                # loaded states invalidate a cached compute() result (the reference, S/metric.py:873-890, would keep
                # returning the value of the states that were replaced)
                self._computed = None
        super()._load_from_state_dict(state_dict, prefix, local_metadata, True, missing_keys, unexpected_keys, error_msgs)

    def _filter_kwargs(self, **kwargs: Any) -> Dict[str, Any]:
        """Keep only the kwargs that ``update`` accepts (all of them if it takes ``**kwargs``)."""
        var_kinds = (inspect.Parameter.VAR_POSITIONAL, inspect.Parameter.VAR_KEYWORD)
        params = self._update_signature.parameters
        filtered = {k: v for k, v in kwargs.items() if k in params and params[k].kind not in var_kinds}
        has_var_kw = any(v.kind == inspect.Parameter.VAR_KEYWORD for v in params.values())
        if not filtered and not has_var_kw:
            return {}
        if has_var_kw:
            return kwargs
        return filtered

    def __hash__(self) -> int:
        vals: List[Any] = [self.__class__.__name__, id(self)]
        for key in self._defaults:
            v = getattr(self, key)
            if hasattr(v, "__iter__") and not isinstance(v, Tensor):
                vals.extend(v)
            else:
                vals.append(v)
        return hash(tuple(vals))

    # -------------------------------------------------------------------------------------------- operator algebra
    def __add__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.add, self, other)

    def __and__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_and, self, other)

    def __eq__(self, other: Any) -> "CompositionalMetric":  # type: ignore[override]
        return CompositionalMetric(torch.eq, self, other)

    def __floordiv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.floor_divide, self, other)

    def __ge__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.ge, self, other)

    def __gt__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.gt, self, other)

    def __le__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.le, self, other)

    def __lt__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.lt, self, other)

    def __matmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.matmul, self, other)

    def __mod__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.fmod, self, other)

    def __mul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.mul, self, other)

    def __ne__(self, other: Any) -> "CompositionalMetric":  # type: ignore[override]
        return CompositionalMetric(torch.ne, self, other)

    def __or__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_or, self, other)

    def __pow__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.pow, self, other)

    def __radd__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.add, other, self)

    def __rand__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_and, self, other)

    def __rfloordiv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.floor_divide, other, self)

    def __rmatmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.matmul, other, self)

    def __rmod__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.fmod, other, self)

    def __rmul__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.mul, other, self)

    def __ror__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_or, other, self)

    def __rpow__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.pow, other, self)

    def __rsub__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.sub, other, self)

    def __rtruediv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.true_divide, other, self)

    def __rxor__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_xor, other, self)

    def __sub__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.sub, self, other)

    def __truediv__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.true_divide, self, other)

    def __xor__(self, other: Any) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_xor, self, other)

    def __abs__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.abs, self, None)

    def __inv__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.bitwise_not, self, None)

    def __invert__(self) -> "CompositionalMetric":
        return self.__inv__()

    def __neg__(self) -> "CompositionalMetric":
        return CompositionalMetric(_neg, self, None)

    def __pos__(self) -> "CompositionalMetric":
        return CompositionalMetric(torch.abs, self, None)

    def __getitem__(self, idx: int) -> "CompositionalMetric":
        return CompositionalMetric(lambda x: x[idx], self, None)

    def __getnewargs__(self) -> Tuple:
        return (Metric.__str__(self),)

    __iter__ = None


def _neg(x: Tensor) -> Tensor:
    return -torch.abs(x)


class CompositionalMetric(Metric):
    """``op(metric_a.compute(), metric_b.compute())``; children sync themselves (reference ``S/metric.py:1088``)."""

    def __init__(
        self,
        operator: Callable,
        metric_a: Union[Metric, builtins.float, Tensor],
        metric_b: Union[Metric, builtins.float, Tensor, None],
    ) -> None:
        super().__init__()
        self.op = operator
        if isinstance(metric_a, Tensor):
            self.register_buffer("metric_a", metric_a, persistent=False)
        else:
            self.metric_a = metric_a
        if isinstance(metric_b, Tensor):
            self.register_buffer("metric_b", metric_b, persistent=False)
        else:
            self.metric_b = metric_b

    def _sync_dist(self, dist_sync_fn: Optional[Callable] = None, process_group: Optional[Any] = None) -> None:
        """Children sync in their own ``compute``."""

    def update(self, *args: Any, **kwargs: Any) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.update(*args, **self.metric_a._filter_kwargs(**kwargs))
        if isinstance(self.metric_b, Metric):
            self.metric_b.update(*args, **self.metric_b._filter_kwargs(**kwargs))

    def compute(self) -> Any:
        val_a = self.metric_a.compute() if isinstance(self.metric_a, Metric) else self.metric_a
        val_b = self.metric_b.compute() if isinstance(self.metric_b, Metric) else self.metric_b
        if val_b is None:
            return self.op(val_a)
        return self.op(val_a, val_b)

    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Any:
        val_a = (
            self.metric_a(*args, **self.metric_a._filter_kwargs(**kwargs))
            if isinstance(self.metric_a, Metric)
            else self.metric_a
        )
        val_b = (
            self.metric_b(*args, **self.metric_b._filter_kwargs(**kwargs))
            if isinstance(self.metric_b, Metric)
            else self.metric_b
        )
        if val_a is None:
            self._forward_cache = None
        elif val_b is None:
            self._forward_cache = None if isinstance(self.metric_b, Metric) else self.op(val_a)
        else:
            self._forward_cache = self.op(val_a, val_b)
        return self._forward_cache

    def reset(self) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.reset()
        if isinstance(self.metric_b, Metric):
            self.metric_b.reset()

    def persistent(self, mode: bool = False) -> None:
        if isinstance(self.metric_a, Metric):
            self.metric_a.persistent(mode=mode)
        if isinstance(self.metric_b, Metric):
            self.metric_b.persistent(mode=mode)

    def __repr__(self) -> str:
        name = self.op.__name__ if hasattr(self.op, "__name__") else repr(self.op)
        return self.__class__.__name__ + f"(\n  {name}(\n    {self.metric_a!r},\n    {self.metric_b!r}\n  )\n)"

    def _wrap_compute(self, compute: Callable) -> Callable:
        return compute


__all__ = ["Metric", "CompositionalMetric", "jit_distributed_available"]
