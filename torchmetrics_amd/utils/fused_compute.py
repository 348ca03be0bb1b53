"""Eager one-launch ``MetricCollection.compute()`` (no HIP graph).

The reference computes a collection member by member (``S/collections.py:310-359``): every member runs its own
``compute()`` -- for the stat-score / confusion-matrix / binned-curve / streaming-regression families a chain of small
ATen ops each (here: one small reduction kernel each, plus 7-36 us of Python per member).

A :class:`CollectionPlan` records, once, the reductions those members' ``compute()`` performs as task descriptors of the
one-launch task kernel (``ops.fused_compute`` -> ``csrc/common/compute_tasks.hip``), and checks per member that this is
ALL its compute does:

* the recorded compute, with its outputs poisoned until the task kernel has run, returns exactly the eager result
  (so the result is the task outputs, or views of them);
* every task input is one of the member's own states (so replaying the tasks needs no other eager op);
* every device-side check the compute defers (``utils/deferred.py``: e.g. AUROC's "nan class" warning) tests a task
  output.

Each later ``compute()`` then re-points the descriptor rows at the members' current states (after a sync, a reset,
``.to()`` ...), points the outputs into one fresh buffer per dtype, runs ONE task-kernel launch, and hands out the
results as views of those buffers; their deferred checks join the collection's one status read.  Members that do not
qualify (list states, host-side computes, custom sync) keep their eager ``compute()``.

The plan is rebuilt when the collection's members change (``add_metrics``), when a fused member's configuration or
device / dtype changes (``Metric._cfg_version``), or when a state's shape / dtype no longer matches the recording.
``TORCHMETRICS_AMD_FUSED_COMPUTE=0`` turns it off.
"""
import operator
import os
import sys
import warnings
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from torchmetrics_amd import ops
from torchmetrics_amd.utils import deferred as _deferred
from torchmetrics_amd.utils.graphs import _leaves, _rebuild, _same_result

# descriptor row layout (ops._TaskRecorder.add): type, blocks, 6 ints, 2 float bit patterns, then the 8 pointer slots
_PTR_COL = 10


def enabled() -> bool:
    return os.environ.get("TORCHMETRICS_AMD_FUSED_COMPUTE", "1") != "0" and torch.cuda.is_available()


class _Member:
    __slots__ = ("key", "metric", "spec", "leaves", "checks", "version")

    def __init__(self, key: str, metric: Any, spec: Any, leaves: List[Tuple[int, torch.dtype, Tuple[int, ...],
                                                                           Tuple[int, ...], int]],
                 checks: List[Tuple[int, str, Any]], version: int) -> None:
        self.key, self.metric, self.spec, self.leaves, self.checks = key, metric, spec, leaves, checks
        self.version = version


class CollectionPlan:
    """The fused part of one collection's ``compute()`` (see the module docstring)."""

    def __init__(self, members: List[Tuple[str, Any]]) -> None:
        self.fused: List[_Member] = []
        self.keys: set = set()
        self.rows: Optional[Tensor] = None
        self.lds = 0
        self.ok = False
        self.state_sig: List[Tuple[Any, str, Tuple[int, ...], torch.dtype]] = []
        self._seen: Optional[Tuple[Any, ...]] = None  # the state objects valid() last checked in full
        self._last_ptrs: Optional[Tuple[int, ...]] = None
        self._same = False
        self._reuse: Optional["_Outputs"] = None
        self._ver_keys: Optional[tuple] = None
        self._build(members)

    # ------------------------------------------------------------------------------------------------- record
    @staticmethod
    def _candidate(m: Any) -> bool:
        from torchmetrics_amd.metric import CompositionalMetric, Metric

        if not isinstance(m, Metric) or isinstance(m, CompositionalMetric) or not m._defaults:
            return False
        for a in m._defaults:
            v = m.__dict__.get(a)
            if not isinstance(v, Tensor) or not v.is_cuda or v.layout != torch.strided:
                return False
        return True

    def _record(self, m: Any):
        """(eager result, recorded result, recorder rows / meta, deferred checks) of one member, or None."""
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            with _deferred.defer():
                eager = type(m).compute(m)
            with ops.fused_compute(poison=True) as rec, _deferred.defer() as dfr:
                recorded = type(m).compute(m)
            rows, meta, lds = list(rec.rows), list(rec.meta), rec.lds
            if not rows:
                return None
            rec.flush()
        return eager, recorded, rows, meta, lds, dfr.items

    def _build(self, members: List[Tuple[str, Any]]) -> None:
        rows_all: List[List[int]] = []
        self.in_slots: List[Tuple[int, Any, str, int]] = []  # (flat index into rows, metric, state, byte offset)
        out_slots: Dict[torch.dtype, List[Tuple[int, int]]] = {}  # dtype -> [(flat index, element offset)]
        out_sizes: Dict[torch.dtype, int] = {}
        self.state_sig: List[Tuple[Any, str, Tuple[int, ...], torch.dtype]] = []
        for key, m in members:
            if not self._candidate(m):
                continue
            try:
                got = self._record(m)
            except Exception:  # noqa: BLE001 - a compute that cannot be recorded stays eager
                got = None
            if got is None:
                continue
            eager, recorded, rows, meta, lds, checks = got
            if not _same_result(_squeeze(eager), _squeeze(recorded)):
                continue
            states = {a: m.__dict__[a] for a in m._defaults}
            spans = {a: t.numel() * t.element_size() for a, t in states.items()}
            # classify every pointer slot: a task output (-> fresh buffer at replay) or one of this member's states
            outs: Dict[int, Tuple[Tensor, int]] = {}  # id(out tensor) -> (tensor, index in local list)
            local_outs: List[Tensor] = []
            member_in: List[Tuple[int, int, str, int]] = []
            member_out: List[Tuple[int, int, int]] = []  # (row, col, local out index)
            good = True
            for r, (tensors, row_outs) in enumerate(meta):
                out_ids = {id(o) for o in row_outs}
                for j, t in enumerate(tensors):
                    if t is None:
                        continue
                    col = _PTR_COL + j  # pointer slot j of the descriptor row
                    if id(t) in out_ids:
                        if id(t) not in outs:
                            outs[id(t)] = (t, len(local_outs))
                            local_outs.append(t)
                        member_out.append((r, col, outs[id(t)][1]))
                        continue
                    ptr = t.data_ptr()
                    hit = None
                    for a, st in states.items():
                        if st.data_ptr() <= ptr < st.data_ptr() + spans[a] and st.is_contiguous():
                            hit = (a, ptr - st.data_ptr())
                            break
                    if hit is None:
                        good = False  # a temporary computed eagerly inside compute(): not replayable
                        break
                    member_in.append((r, col, hit[0], hit[1]))
                if not good:
                    break
            if not good or any(not o.is_contiguous() for o in local_outs):
                continue
            # result leaves must be views of the task outputs
            leaves: List[Tensor] = []
            spec = _leaves(_squeeze(recorded), leaves)
            leaf_info = []
            for leaf in leaves:
                src = next((o for o in local_outs if o.untyped_storage().data_ptr() == leaf.untyped_storage().data_ptr()),
                           None)
                if src is None or leaf.dtype != src.dtype:
                    good = False
                    break
                leaf_info.append((local_outs.index(src), leaf.dtype, tuple(leaf.shape), tuple(leaf.stride()),
                                  leaf.storage_offset() - src.storage_offset()))
            chk = []
            for flag, msg, exc in checks:
                src = next((i for i, o in enumerate(local_outs) if o.dtype == flag.dtype and flag.numel() == 1
                            and o.data_ptr() <= flag.data_ptr() < o.data_ptr() + o.numel() * o.element_size()), None)
                if src is None:
                    good = False
                    break
                rel = (flag.data_ptr() - local_outs[src].data_ptr()) // flag.element_size()
                chk.append((src, rel, msg, exc))
            if not good:
                continue
            # commit this member: its rows / slots join the plan; its outputs get offsets in the per-dtype buffers
            base_row = len(rows_all)
            out_off = []
            for o in local_outs:
                off = out_sizes.get(o.dtype, 0)
                out_off.append((o.dtype, off))
                out_sizes[o.dtype] = off + o.numel()
            ncol = len(rows[0])
            for r, c, a, boff in member_in:
                self.in_slots.append(((base_row + r) * ncol + c, m, a, boff))
            for r, c, li in member_out:
                dt, off = out_off[li]
                out_slots.setdefault(dt, []).append(((base_row + r) * ncol + c, off))
            rows_all.extend(rows)
            self.lds = max(self.lds, lds)
            self.state_sig.extend((m, a, tuple(t.shape), t.dtype) for a, t in states.items())
            glob_leaves = [(out_off[li][0], out_off[li][1] + rel, shape, stride)
                           for li, _dt, shape, stride, rel in leaf_info]
            glob_checks = [(out_off[li][0], out_off[li][1] + rel, msg, exc) for li, rel, msg, exc in chk]
            self.fused.append(_Member(key, m, spec, glob_leaves, glob_checks, m.__dict__.get("_cfg_version", 0)))
        if not self.fused:
            return
        self.rows = torch.tensor(rows_all, dtype=torch.int64)
        self.flat_np = self.rows.numpy().reshape(-1)  # the same memory: pointer patches go through numpy (~1 us each)
        self.ncol = self.rows.shape[1]
        # every output dtype's buffer is a 256-byte aligned piece of ONE byte allocation per run
        self.out_layout: List[Tuple[torch.dtype, int, int]] = []  # (dtype, byte offset, bytes)
        nbytes = 0
        for dt, n in out_sizes.items():
            nb = n * torch.empty(0, dtype=dt).element_size()
            self.out_layout.append((dt, nbytes, nb))
            nbytes += -(-nb // 256) * 256
        self.out_bytes_total = max(nbytes, 256)
        base = {dt: off for dt, off, _ in self.out_layout}
        self.out_idx = np.array([i for sl in out_slots.values() for i, _ in sl], dtype=np.int64)
        self.out_rel = np.array([base[dt] + o * torch.empty(0, dtype=dt).element_size()
                                 for dt, sl in out_slots.items() for _, o in sl], dtype=np.int64)
        self.in_idx = np.array([i for i, _, _, _ in self.in_slots], dtype=np.int64)
        self.in_off = np.array([o for _, _, _, o in self.in_slots], dtype=np.int64)
        # distinct (metric, state) pairs, in slot order, and each slot's index into them
        pairs: Dict[Tuple[int, str], int] = {}
        self.in_pairs: List[Tuple[Any, str]] = []
        slot_pair = []
        for _, m, a, _ in self.in_slots:
            k = (id(m), a)
            if k not in pairs:
                pairs[k] = len(self.in_pairs)
                self.in_pairs.append((m, a))
            slot_pair.append(pairs[k])
        self.slot_pair = np.array(slot_pair, dtype=np.int64)
        self.keys = {f.key for f in self.fused}
        self.device = self.fused[0].metric.__dict__[self.in_pairs[0][1]].device if self.in_pairs else None
        self.ok = self.device is not None

    # ------------------------------------------------------------------------------------------------- replay
    def valid(self) -> bool:
        ver = self._ver_keys
        if ver is None:
            ver = self._ver_keys = ([f.metric.__dict__ for f in self.fused], [f.version for f in self.fused],
                                    [m.__dict__ for m, _, _, _ in self.state_sig], [a for _, a, _, _ in self.state_sig])
        for d, v in zip(ver[0], ver[1]):
            if d.get("_cfg_version", 0) != v:
                return False
        # the same state objects as at the last full check (the common case: states updated in place): valid, and
        # their memory has not moved (run() keeps the pointers it patched last time)
        cur = list(map(dict.get, ver[2], ver[3]))
        seen = self._seen
        if seen is not None and len(cur) == len(seen) and all(map(operator.is_, cur, seen)):
            self._same = True
            return True
        self._same = False
        for (m, a, shape, dtype), t in zip(self.state_sig, cur):
            if not isinstance(t, Tensor) or t.dtype != dtype or t.shape != shape or not t.is_cuda:
                return False
        self._seen = cur
        return True

    def run(self) -> Tuple[Dict[str, Any], Dict[str, List[Tuple[Tensor, str, Any]]]]:
        """One launch for every fused member: ``({key: result}, {key: deferred checks})``.

        The output buffer and the result views of the last run are reused when nothing outside this plan still
        refers to them (every view object back at the reference count it had when built, and no other tensor on
        the buffer's storage): a per-step ``compute()`` whose results were logged and dropped then costs one launch
        and no view construction (13 ``as_strided`` views were ~20 us of host time per compute of config #5).  A
        result the caller kept -- or a member's cached ``compute()`` value -- makes the plan build a fresh buffer, so
        a handed-out result never changes."""
        flat = self.flat_np
        if not (self._same and self._last_ptrs is not None):
            ptrs = tuple(m.__dict__[a].data_ptr() for m, a in self.in_pairs)
            if ptrs != self._last_ptrs:  # states moved (reset, sync, .to()): re-point the input slots
                flat[self.in_idx] = np.asarray(ptrs, dtype=np.int64)[self.slot_pair] + self.in_off
                self._last_ptrs = ptrs
        c = self._reuse
        if c is None or not c.idle():
            raw = torch.empty(self.out_bytes_total, dtype=torch.uint8, device=self.device)
            flat[self.out_idx] = self.out_rel + raw.data_ptr()
            bufs = {dt: raw[off : off + nb].view(dt) for dt, off, nb in self.out_layout}
            strided = torch.as_strided
            leaves: List[List[Tensor]] = []
            checks: Dict[str, List[Tuple[Tensor, str, Any]]] = {}
            for f in self.fused:
                # (as_strided offsets count from the shared storage's start: add each dtype view's own offset)
                leaves.append([strided(bufs[dt], shape, stride, bufs[dt].storage_offset() + off)
                               for dt, off, shape, stride in f.leaves])
                if f.checks:
                    checks[f.key] = [(bufs[dt][off : off + 1], msg, exc) for dt, off, msg, exc in f.checks]
            # the results too are built once per buffer: reused with it (a results mapping or container held outside
            # holds its leaves, so idle() sees it)
            results = {f.key: _rebuild(f.spec, lv) for f, lv in zip(self.fused, leaves)}
            c = self._reuse = _Outputs(raw, bufs, leaves, checks, results)
        tasks = ops._ops().compute_tasks
        mx = 32
        for i in range(0, self.rows.shape[0], mx):
            tasks(self.rows[i : i + mx], c.raw, self.lds)
        return c.results, c.checks


class _Outputs:
    """One run's output buffer and the views handed out from it, with the reference counts they have while only
    the plan holds them (see :meth:`CollectionPlan.run`)."""

    __slots__ = ("raw", "bufs", "leaves", "checks", "results", "storage", "use", "rc")

    def __init__(self, raw: Tensor, bufs: Dict[torch.dtype, Tensor], leaves: List[List[Tensor]],
                 checks: Dict[str, List[Tuple[Tensor, str, Any]]], results: Dict[str, Any]) -> None:
        self.raw, self.bufs, self.leaves, self.checks, self.results = raw, bufs, leaves, checks, results
        self.storage = raw.untyped_storage()
        self.use = torch._C._storage_Use_Count(self.storage._cdata)
        # (counted the way idle() counts: the list's reference + the call's argument, no loop variable / zip tuple)
        self.rc = [[sys.getrefcount(lv[i]) for i in range(len(lv))] for lv in leaves]

    def idle(self) -> bool:
        if torch._C._storage_Use_Count(self.storage._cdata) != self.use:
            return False  # another tensor on the buffer (a view of a result, a check slice kept alive ...)
        getrc = sys.getrefcount
        for lv, rc in zip(self.leaves, self.rc):
            for i in range(len(lv)):
                if getrc(lv[i]) != rc[i]:
                    return False  # a result (or a member's cached compute() value) is still held
        return True


def _squeeze(v: Any) -> Any:
    from torchmetrics_amd.utilities.data import _squeeze_if_scalar

    return _squeeze_if_scalar(v)


__all__ = ["CollectionPlan", "enabled"]
