"""``MetricCollection`` with compute groups and collection-level (sync-once) distributed sync.

API/behaviour parity with reference ``S/collections.py:34-661`` (kwargs filtering, prefix/postfix, nested
collections, compute groups discovered on the first ``update`` and shared by reference, ``copy_state`` semantics).

MI355X-first change -- **one sync per collection**: the reference ``compute`` calls every member's ``compute``, and
each one syncs its own states (``S/collections.py:330-338``), i.e. per state 1 barrier + 2 all_gathers, repeated for
every member even when compute groups share the states.  Here ``compute`` syncs the *group leaders* of all eligible
members in ONE engine call (:func:`torchmetrics_amd.parallel.sync.sync_state_dicts`): for a 20-metric
classification+regression collection that is one ``all_reduce`` per (op, dtype) bucket -- typically 2-3 RCCL
collectives in total.  Every member's ``compute()`` still returns the synced value and local states are restored
afterwards, exactly like the per-metric path.
"""
import operator
from itertools import repeat
from collections import OrderedDict
from copy import deepcopy
from typing import Any, Dict, Hashable, Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import ModuleDict

from torchmetrics_amd import ops
from torchmetrics_amd.metric import CompositionalMetric, Metric, jit_distributed_available
from torchmetrics_amd.parallel.sync import distributed_available as _engine_dist_available
from torchmetrics_amd.parallel import arena as _arena
from torchmetrics_amd.parallel.sync import sync_state_dicts
from torchmetrics_amd.utilities.data import _flatten_dict, allclose
from torchmetrics_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE, plot_single_or_multi_val
from torchmetrics_amd.utilities.prints import rank_zero_warn
from torchmetrics_amd.utils import deferred as _deferred
from torchmetrics_amd.utils import profiling as _prof
from torchmetrics_amd.utils import validation as _validation
from torchmetrics_amd.utils.deferred import WORD_CODES as _WORD_CODES


class MetricCollection(ModuleDict):
    """Chain metrics that take the same inputs into one ``update``/``compute``/``forward``.

    Args:
        metrics: a metric, a sequence of metrics, or a dict ``name -> metric``; nested collections are flattened.
        additional_metrics: more metrics when ``metrics`` is a metric/sequence.
        prefix / postfix: strings added around every output key.
        compute_groups: ``True`` (auto-detect metrics with identical states after the first update), ``False``, or an
            explicit list of lists of metric names.
    """

    _modules: Dict[str, Metric]  # type: ignore[assignment]
    _groups: Dict[int, List[str]]

    def __init__(
        self,
        metrics: Union[Metric, Sequence[Metric], Dict[str, Metric]],
        *additional_metrics: Metric,
        prefix: Optional[str] = None,
        postfix: Optional[str] = None,
        compute_groups: Union[bool, List[List[str]]] = True,
    ) -> None:
        super().__init__()
        self.prefix = self._check_arg(prefix, "prefix")
        self.postfix = self._check_arg(postfix, "postfix")
        self._enable_compute_groups = compute_groups
        self._groups_checked: bool = False
        self._state_is_copy: bool = False
        self.add_metrics(metrics, *additional_metrics)

    # ------------------------------------------------------------------------------------------------ hot path
    @torch.jit.unused
    def forward(self, *args: Any, **kwargs: Any) -> Dict[str, Any]:
        return self._compute_and_reduce("forward", *args, **kwargs)

    def update(self, *args: Any, **kwargs: Any) -> None:
        """Update every metric (only the first member of each compute group once groups are known)."""
        if self._groups_checked or not self._enable_compute_groups:
            d = self.__dict__
            nc = d.get("_names_cache")
            if nc is None or nc[0] is not d["_groups"] or nc[1] != self._groups_checked:
                names = [cg[0] for cg in self._groups.values()] if self._groups_checked else list(self._modules.keys())
                nc = d["_names_cache"] = (d["_groups"], self._groups_checked, names,
                                          tuple(id(self._modules[n]) for n in names))
            names = nc[2]
            # few-class multiclass leaders on the same (preds, target): ONE fused pass for all of them
            # (utils/fused_update.py, csrc/classification/family.hip)
            done = self._fused_update(names, args, kwargs)
            # a step the streaming regression leaders already merged into one moments call is replayed directly
            # (utils/fused_moments.py): no per-member update wrappers, checks and plan objects
            replayed = self._replay_moments(args, kwargs)
            # streaming regression leaders hand their moments requests to `sink`; requests on the same inputs are
            # then merged into one kernel pass for the whole collection (ops.run_moments_plans)
            sink: list = []
            submitted: list = []
            modules = self._modules
            for name in names:
                m0 = modules[name]
                if (done and id(m0) in done) or (replayed and id(m0) in replayed):
                    continue
                d = m0.__dict__
                d["_moments_sink"] = sink
                n0 = len(sink)
                try:
                    m0.update(*args, **m0._filter_kwargs(**kwargs))
                finally:
                    del d["_moments_sink"]
                if len(sink) == n0 + 1:
                    submitted.append(m0)
            if sink:
                merged: list = []
                ops.run_moments_plans(sink, merged)
                if not replayed and not kwargs and len(args) == 2:
                    from torchmetrics_amd.utils import fused_moments as _fm

                    self.__dict__["_moments_replay"] = _fm.build(submitted, merged, len(sink), args[0], args[1])
            if self._state_is_copy and self._groups_checked:
                self._compute_groups_create_state_ref()
                self._state_is_copy = False
        else:
            for m in self.values(copy_state=False):
                m.update(*args, **m._filter_kwargs(**kwargs))
            if self._enable_compute_groups:
                self._merge_compute_groups()
                self._compute_groups_create_state_ref()
                self._groups_checked = True

    def _replay_moments(self, args: tuple, kwargs: dict) -> Optional[set]:
        """Replay the recorded merged regression call (utils/fused_moments.py); returns the ids of the members it
        updated, or None (and the record is dropped when it no longer applies)."""
        rp = self.__dict__.get("_moments_replay")
        if rp is None or kwargs or len(args) != 2:
            return None
        from torchmetrics_amd.utils import validation as _validation

        if _validation.STRICT or not rp.run(args[0], args[1]):
            self.__dict__["_moments_replay"] = None
            return None
        return rp.member_ids

    def _fused_update(self, names: List[str], args: tuple, kwargs: dict) -> Optional[set]:
        """Run the fused few-class multiclass update (utils/fused_update.py) for the leaders it serves; returns the
        ids of the metrics it updated (None: nothing fused)."""
        if kwargs or len(args) != 2 or not isinstance(args[0], Tensor) or not args[0].is_cuda:
            return None
        from torchmetrics_amd.utils import fused_update as _fu
        from torchmetrics_amd.utils import validation as _validation

        if _validation.STRICT:  # the reference's per-update raises: every member validates on its own
            return None

        d = self.__dict__
        nc = d.get("_names_cache")
        ident = nc[3] if nc is not None and nc[2] is names else tuple(id(self._modules[n]) for n in names)
        entry = d.get("_family_plan")
        if entry is None or entry[0] != ident or not entry[1].valid(None):
            entry = (ident, _fu.FamilyPlan([(n, self._modules[n]) for n in names]))
            d["_family_plan"] = entry
        plan = entry[1]
        if not plan.ok or not plan.run(args[0], args[1]):
            return None
        return plan.metric_ids

    def _merge_compute_groups(self) -> None:
        """Merge groups whose leaders hold identical states (O(M^2) pairwise, once)."""
        changed = True
        while changed:
            changed = False
            keys = list(self._groups.keys())
            for i, a in enumerate(keys):
                for b in keys[i + 1 :]:
                    if a not in self._groups or b not in self._groups:
                        continue
                    m1 = getattr(self, self._groups[a][0])
                    m2 = getattr(self, self._groups[b][0])
                    if self._equal_metric_states(m1, m2):
                        self._groups[a].extend(self._groups.pop(b))
                        changed = True
        self._groups = dict(enumerate(self._groups.values()))

    @staticmethod
    def _equal_metric_states(metric1: Metric, metric2: Metric) -> bool:
        if len(metric1._defaults) == 0 or len(metric2._defaults) == 0:
            return False
        if metric1._defaults.keys() != metric2._defaults.keys():
            return False
        for key in metric1._defaults:
            s1, s2 = getattr(metric1, key), getattr(metric2, key)
            if type(s1) != type(s2):  # noqa: E721
                return False
            if isinstance(s1, Tensor) and isinstance(s2, Tensor):
                return s1.shape == s2.shape and allclose(s1, s2)
            if isinstance(s1, list) and isinstance(s2, list):
                return all(a.shape == b.shape and allclose(a, b) for a, b in zip(s1, s2))
        return True

    def _compute_groups_create_state_ref(self, copy: bool = False) -> None:
        """Point every group member's states at the leader's (or deep-copy them when ``copy``)."""
        # called by every items() / values() / [] access: plain attributes go straight to __dict__ (they live there;
        # nn.Module.__setattr__ costs ~1 us per call), states through setattr only when a reference is stale
        d = self.__dict__
        if not d["_state_is_copy"] and not copy:
            # steady state: every follower already holds its leader's state objects -- one C-speed identity pass over
            # flattened (leader, follower, state) lists built once per groups object (the per-state walk below was
            # ~6 us per compute() of config #5)
            groups = d.get("_groups")
            fast = d.get("_ref_fast")
            if fast is None or fast[0] is not groups:
                fast = d["_ref_fast"] = (groups, *self._ref_fast_lists())
            _, lead_d, foll_d, names, pairs = fast
            lv = list(map(dict.get, lead_d, names))
            if not any(map(operator.is_, lv, repeat(None))) and all(map(operator.is_, map(dict.get, foll_d, names), lv)):
                for d0, di in pairs:
                    di["_update_count"] = d0["_update_count"]
                    if d0["_computed"] is None:
                        di["_computed"] = None
                return
        if not d["_state_is_copy"]:
            modules = self._modules
            for cg in self._groups.values():
                if len(cg) == 1:
                    continue
                m0 = modules[cg[0]]
                d0 = m0.__dict__
                cur = [(s, d0[s] if s in d0 else getattr(m0, s)) for s in m0._defaults]
                for name in cg[1:]:
                    mi = modules[name]
                    di = mi.__dict__
                    for state, val in cur:
                        if copy:
                            setattr(mi, state, deepcopy(val))
                        elif di.get(state, None) is not val and getattr(mi, state) is not val:
                            setattr(mi, state, val)
                    di["_update_count"] = d0["_update_count"]
                    # members share the leader's *states*, not its result: only propagate cache invalidation (the
                    # reference copies the leader's cached value, so a second compute() without an update returned
                    # the leader's result for every member, S/collections.py:307)
                    if copy:
                        di["_computed"] = deepcopy(di["_computed"])
                    elif d0["_computed"] is None:
                        di["_computed"] = None
        d["_state_is_copy"] = copy

    def _ref_fast_lists(self) -> Tuple[List[dict], List[dict], List[str], List[Tuple[dict, dict]]]:
        """(leader dicts, follower dicts, state names) flattened over every (follower, state) of the compute groups,
        and the (leader dict, follower dict) pairs."""
        lead_d: List[dict] = []
        foll_d: List[dict] = []
        names: List[str] = []
        pairs: List[Tuple[dict, dict]] = []
        modules = self._modules
        for cg in self._groups.values():
            if len(cg) == 1 or any(n not in modules for n in cg):
                continue
            d0 = modules[cg[0]].__dict__
            states = list(modules[cg[0]]._defaults)
            for name in cg[1:]:
                di = modules[name].__dict__
                pairs.append((d0, di))
                for st in states:
                    lead_d.append(d0)
                    foll_d.append(di)
                    names.append(st)
        return lead_d, foll_d, names, pairs

    def compute(self) -> Dict[str, Any]:
        if _prof.ENABLED:
            with _prof.range("tm.collection.compute"):
                return self._compute_and_reduce("compute")
        return self._compute_and_reduce("compute")

    # ----------------------------------------------------------------------------------------- sync-once engine
    def _eligible_for_collection_sync(self, m: Metric) -> bool:
        return (
            isinstance(m, Metric)
            and not isinstance(m, CompositionalMetric)
            and type(m)._sync_dist is Metric._sync_dist
            and m.dist_sync_fn is None
            and m._to_sync
            and not m._is_synced
            and m._computed is None
            and bool(m.distributed_available_fn() if callable(m.distributed_available_fn) else False)
        )

    def _collection_sync(self) -> List[Tuple[Metric, bool]]:
        """Sync all eligible members with one engine call; returns ``(metric, saved _to_sync)`` to restore."""
        if not _engine_dist_available() and all(
                m.__dict__.get("distributed_available_fn") is jit_distributed_available for m in self._modules.values()):
            return []  # one process: nothing to sync (no per-member eligibility walk)
        members = dict(self.items(keep_base=True, copy_state=False))
        if self._groups:
            groups = [cg for cg in self._groups.values()]
            covered = {n for cg in groups for n in cg}
            groups += [[n] for n in members if n not in covered]
        else:
            groups = [[n] for n in members]
        plans: Dict[Any, List[List[Metric]]] = {}
        for cg in groups:
            ms = [members[n] for n in cg if n in members]
            if not ms or not all(self._eligible_for_collection_sync(m) for m in ms):
                continue
            key = id(ms[0].process_group) if ms[0].process_group is not None else None
            plans.setdefault(key, []).append(ms)
        restore: List[Tuple[Metric, bool]] = []
        for _, grp_list in plans.items():
            leaders = [g[0] for g in grp_list]
            # every leader's reducible states in ONE arena per (reduction, dtype, device), in the engine's bucket order:
            # each bucket of this sync is then one span (no-op once laid out); followers re-point to the views
            if not _arena.is_packed(leaders):
                _arena.pack(leaders)
                for g in grp_list:
                    for m in g[1:]:
                        for a in g[0]._defaults:
                            m.__dict__[a] = g[0].__dict__[a]
            # a member whose compute() needs less than its states syncs that instead (calibration: its bins as a SUM
            # bucket of this same engine call, not its sample lists); fixed-shape gather states go signed, headerless
            overrides = [m._compute_sync_override() for m in leaders]
            entries = [ov if ov is not None else ({a: getattr(m, a) for a in m._reductions}, m._reductions,
                                                   m._static_gather_spec())
                       for m, ov in zip(leaders, overrides)]
            word = self._sync_word(entries)
            # overflowed narrow buckets / failed static signatures land in the word too (NARROW_RETRY): no host read
            # in the sync, the collection's one validation read sees them and re-syncs
            synced = sync_state_dicts(entries, group=leaders[0].process_group, err_word=word, narrow_word=word)
            for g, states, ov in zip(grp_list, synced, overrides):
                for m in g:
                    m._cache = {a: getattr(m, a) for a in m._defaults}
                    if ov is not None:
                        m._compute_sync_finish(states)
                    else:
                        for a, v in states.items():
                            setattr(m, a, v)
                    m._is_synced = True
                    restore.append((m, m._to_sync))
                    m._to_sync = False
        return restore

    def _sync_word(self, entries: List[Tuple[Dict[str, Any], Dict[str, Any]]]) -> Optional[Tensor]:
        """The collection's int32 status word for the one-shot buckets of its one engine call (``None`` off-GPU)."""
        dev = next((v.device for e in entries for v in e[0].values() if isinstance(v, Tensor) and v.is_cuda), None)
        if dev is None:
            return None
        d = self.__dict__
        word = d.get("_oneshot_word")
        if word is None or word.device != dev:
            word = torch.zeros(1, dtype=torch.int32, device=dev)
            d["_oneshot_word"] = word
        d["_oneshot_word_pending"] = True
        return word

    def _defer_device_checks(self) -> Optional[Tuple[Optional[Tensor], List[Metric]]]:
        """Before the members' computes: mark every member whose ROCm validation word is unread as provisionally
        clean (its own ``compute()`` then skips its read) -- :meth:`_finish_device_checks` reads all of them, the sync's
        one-shot status and every check the computes deferred (``utils/deferred.py``) with ONE device read."""
        d = self.__dict__
        word = d.get("_oneshot_word") if d.pop("_oneshot_word_pending", False) else None
        pending = []
        for m in self._modules.values():
            md = m.__dict__
            w = md["_device_errors"]
            if w is not None and w.is_cuda and md.get("_errors_checked_at") != md["_update_count"]:
                md["_device_errors_clean"] = True
                pending.append(m)
        if word is None and not pending:
            return None
        return word, pending

    def _finish_device_checks(self, plan: Optional[Tuple[Optional[Tensor], List[Metric]]], items: List[Any]) -> bool:
        """One read of every word; raises what they hold.  True: the sync's word asks for a re-sync (a narrow bucket
        overflowed or a static-shape signature failed -- every rank sees the same verdict), nothing was raised for it
        and the caller syncs and computes again."""
        word, pending = plan if plan is not None else (None, [])
        words: List[Tuple[Tensor, int]] = []
        if word is not None:
            words.append((word, 0))
        words += [(m.__dict__["_device_errors"], 0) for m in pending]
        flags = []
        for flag, msg, exc in items:
            code = _WORD_CODES.get(flag.dtype)
            if code is None:
                flag, code = (flag != 0), 4
            words.append((flag, code))
            flags.append((msg, exc))
        if not words:
            return False
        dev = words[0][0].device
        cached = self.__dict__.get("_word_table1")
        same = (cached is not None and len(cached[2]) == len(words)
                and all(map(operator.is_, cached[2], (w for w, _ in words))))  # (checked on one device before)
        if not same and any(w.device != dev for w, _ in words):
            codes = [int(w.reshape(-1)[0].item()) if c == 0 else int(w.reshape(-1)[0].item() != 0)
                     for w, c in words]  # (several devices: rare, read each)
        else:
            codes = self._read_words(words)
        nw = 1 if word is not None else 0
        if word is not None and codes[0] & _validation.NARROW_RETRY:
            from torchmetrics_amd.parallel.sync import narrow_resolve

            word.bitwise_and_(~_validation.NARROW_RETRY)
            narrow_resolve(word)
            if not codes[0] & ~_validation.NARROW_RETRY:
                return True
        if word is not None and codes[0]:
            self._raise_oneshot(word)
        for m, code in zip(pending, codes[nw : nw + len(pending)]):
            if code:
                m.__dict__.pop("_device_errors_clean", None)
                m._raise_device_errors()  # the member's own message (re-reads its word)
        for m in pending:
            md = m.__dict__
            md["_errors_checked_at"] = md["_update_count"]
        rest = codes[nw + len(pending):]
        for (msg, exc), code in zip(flags, rest):
            if code and exc is not None:
                raise exc(msg)
        for (msg, exc), code in zip(flags, rest):
            if code:
                rank_zero_warn(msg, UserWarning)
        return False

    def __getstate__(self) -> Dict[str, Any]:
        # process-local handles: the mapped pinned status buffer (its device address) and the fused-compute plan
        # (descriptor rows holding device pointers) are rebuilt on first use in the copy
        state = self.__dict__.copy()
        for k in ("_status_host", "_status_ptr", "_fused_plan", "_compute_calls", "_fused_rebuilds", "_fused_off",
                  "_family_plan", "_moments_replay", "_word_tables", "_word_table1", "_ref_fast",
                  "_names_cache", "_ident_cache"):
            state.pop(k, None)
        return state

    def _fused_compute(self, members: List[Tuple[str, Metric]]) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        """The members whose compute() is only fused reductions, in ONE task-kernel launch (utils/fused_compute.py;
        recorded at the second compute() of the collection, re-recorded when its members or their configuration
        change)."""
        from torchmetrics_amd.utils import fused_compute as _fc

        d = self.__dict__
        calls = d.get("_compute_calls", 0)
        d["_compute_calls"] = calls + 1
        if calls == 0 or d.get("_fused_off") or not _fc.enabled():
            return {}, {}
        ic = d.get("_ident_cache")
        if ic is None or ic[0] is not d.get("_groups") or len(ic[1]) != len(members) or not all(
                map(operator.is_, ic[2], (m for _, m in members))):
            ic = d["_ident_cache"] = (d.get("_groups"), tuple(id(m) for _, m in members), [m for _, m in members])
        ident = ic[1]
        plan = d.get("_fused_plan")
        if plan is None or plan[0] != ident or not plan[1].valid():
            rebuilds = d.get("_fused_rebuilds", 0)
            if rebuilds >= 8:  # members whose configuration keeps changing: stay eager
                d["_fused_off"] = True
                return {}, {}
            d["_fused_rebuilds"] = rebuilds + 1
            plan = (ident, _fc.CollectionPlan(members))
            d["_fused_plan"] = plan
        if not plan[1].ok:
            return {}, {}
        return plan[1].run()

    @staticmethod
    def _take_fused(m: Metric, value: Any) -> Any:
        """What the member's compute() wrapper does around a value (Metric._wrap_compute): its cached value if it has
        one, the compute-before-update warning, the cache."""
        d = m.__dict__
        if d["_computed"] is not None:
            return d["_computed"]
        if not d["_update_count"]:
            rank_zero_warn(
                f"The ``compute`` method of metric {m.__class__.__name__}"
                " was called before the ``update`` method which may lead to errors,"
                " as metric states have not yet been updated.",
                UserWarning,
            )
        if d["compute_with_cache"]:
            d["_computed"] = value
        return value

    def _read_words(self, words: List[Tuple[Tensor, int]]) -> List[int]:
        """One kernel writes every word into pinned host memory, the host reads them (no device->host copy): up to 128
        words in ONE native call that spins on a sequence number the kernel stores after the words (no stream-sync
        round trip, ``ops.read_words``), else the gather launch(es) + a stream sync."""
        d = self.__dict__
        if len(words) <= 128:
            # the same word tensors as last time (the steady state): their table is reused without re-reading any
            # data_ptr (a word tensor's storage does not move)
            cached = d.get("_word_table1")
            if (cached is None or len(cached[2]) != len(words)
                    or not all(map(operator.is_, cached[2], (w for w, _ in words)))
                    or cached[3] != [c for _, c in words]):
                key = tuple((w.data_ptr(), c) for w, c in words)
                cached = d["_word_table1"] = (key, torch.tensor([list(k) for k in key], dtype=torch.int64),
                                              [w for w, _ in words], [c for _, c in words])
            fast = ops.read_words(cached[1], words[0][0])
            if fast is not None:
                return fast
        key = tuple((w.data_ptr(), c) for w, c in words)
        host = d.get("_status_host")
        if host is None or host.numel() < len(words):
            host = torch.zeros(max(128, len(words)), dtype=torch.int32, pin_memory=True)
            d["_status_host"] = host
            d["_status_ptr"] = int(ops._ops().mapped_device_ptr(host))
        ptr = d["_status_ptr"]
        # the word table of a steady collection repeats every compute: keep the last one (a host tensor built from
        # a Python list costs more than the gather launch)
        cached = d.get("_word_tables")
        if cached is None or cached[0] != key:
            tables = [torch.tensor([list(k) for k in key[i : i + 128]], dtype=torch.int64)
                      for i in range(0, len(words), 128)]
            cached = d["_word_tables"] = (key, tables)
        for j, table in enumerate(cached[1]):
            ops._ops().gather_words(table, ptr + 4 * 128 * j, words[128 * j][0])
        torch.cuda.current_stream(words[0][0].device).synchronize()
        return host[: len(words)].tolist()

    @staticmethod
    def _raise_oneshot(word: Tensor) -> None:
        code = int(word.item())
        word.zero_()
        _validation.raise_for_code(code)

    def _compute_synced(self, members: List[Tuple[str, Metric]], result: Dict[str, Any]) -> bool:
        """Sync (one engine call), compute every member, then ONE read of every validation word plus the sync's
        status (a rank raising before the collectives would leave its peers waiting in them).  True: the sync must be
        repeated (every rank got the same verdict); the members are un-synced again either way."""
        restore = self._collection_sync()
        try:
            plan = self._defer_device_checks()
            try:
                fused, fchecks = self._fused_compute(members)
                local = not fused or not _engine_dist_available()
                with _deferred.defer() as dfr:
                    items = dfr.items
                    take = self._take_fused
                    for k, m in members:
                        val = fused.get(k) if fused else None
                        if val is not None and (local or m.__dict__["_is_synced"]):
                            md = m.__dict__
                            # (the common case of _take_fused inline: no cached value, updated, cache on)
                            if md["_computed"] is None and md["_update_count"] and md["compute_with_cache"]:
                                md["_computed"] = val
                                result[k] = val
                            else:
                                result[k] = take(m, val)
                            chk = fchecks.get(k)
                            if chk:
                                items.extend(chk)
                        else:
                            result[k] = m.compute()
                return self._finish_device_checks(plan, dfr.items)
            except BaseException:
                for m in self._modules.values():
                    m.__dict__["_computed"] = None  # nothing computed in a failed call is handed out later
                raise
        finally:
            for m in self._modules.values():
                m.__dict__.pop("_device_errors_clean", None)
            for m, to_sync in restore:
                if m._is_synced:
                    m.unsync()
                m._to_sync = to_sync

    def _compute_and_reduce(self, method_name: str, *args: Any, **kwargs: Any) -> Dict[str, Any]:
        result: Dict[str, Any] = {}
        members = list(self.items(keep_base=True, copy_state=False))  # (group members re-pointed once per call)
        if method_name == "compute":
            for _ in range(4):  # a re-sync (narrow overflow / static signature) moves buckets to a safer wire: <= 3
                if not self._compute_synced(members, result):
                    break
                for m in self._modules.values():
                    m.__dict__["_computed"] = None  # values of the discarded sync are not handed out
                result = {}
            else:
                raise RuntimeError("MetricCollection.compute(): the state sync did not settle after 3 re-syncs")
        elif method_name == "forward":
            for k, m in members:
                result[k] = m(*args, **m._filter_kwargs(**kwargs))
        else:
            raise ValueError(f"method_name should be either 'compute' or 'forward', but got {method_name}")

        if not any(isinstance(v, dict) for v in result.values()):
            if self.prefix is None and self.postfix is None:
                return result
            return {self._set_name(k): v for k, v in result.items()}
        _, duplicates = _flatten_dict(result)
        flat: Dict[str, Any] = {}
        for k, m in members:
            res = result[k]
            if isinstance(res, dict):
                for key, v in res.items():
                    if duplicates:
                        stripped = k.replace(getattr(m, "prefix", "") or "", "")
                        stripped = stripped.replace(getattr(m, "postfix", "") or "", "")
                        key = f"{stripped}_{key}"
                    if getattr(m, "_from_collection", None) and m.prefix is not None:
                        key = f"{m.prefix}{key}"
                    if getattr(m, "_from_collection", None) and m.postfix is not None:
                        key = f"{key}{m.postfix}"
                    flat[key] = v
            else:
                flat[k] = res
        return {self._set_name(k): v for k, v in flat.items()}

    # -------------------------------------------------------------------------------------------- management
    def reset(self) -> None:
        for m in self.values(copy_state=False):
            m.reset()
        if self._enable_compute_groups and self._groups_checked:
            self._compute_groups_create_state_ref()

    def clone(self, prefix: Optional[str] = None, postfix: Optional[str] = None) -> "MetricCollection":
        mc = deepcopy(self)
        if prefix:
            mc.prefix = self._check_arg(prefix, "prefix")
        if postfix:
            mc.postfix = self._check_arg(postfix, "postfix")
        return mc

    def persistent(self, mode: bool = True) -> None:
        for m in self.values(copy_state=False):
            m.persistent(mode)

    def add_metrics(
        self, metrics: Union[Metric, Sequence[Metric], Dict[str, Metric]], *additional_metrics: Metric
    ) -> None:
        if isinstance(metrics, Metric):
            metrics = [metrics]
        if isinstance(metrics, Sequence):
            metrics = list(metrics)
            remain: list = []
            for m in additional_metrics:
                (metrics if isinstance(m, Metric) else remain).append(m)
            if remain:
                rank_zero_warn(f"You have passes extra arguments {remain} which are not `Metric` so they will be ignored.")
        elif additional_metrics:
            raise ValueError(
                f"You have passes extra arguments {additional_metrics} which are not compatible"
                f" with first passed dictionary {metrics} so they will be ignored."
            )

        def _absorb(prefix_name: Optional[str], coll: "MetricCollection") -> None:
            for k, v in coll.items(keep_base=False):
                v.postfix = coll.postfix
                v.prefix = coll.prefix
                v._from_collection = True
                self[f"{prefix_name}_{k}" if prefix_name is not None else k] = v

        if isinstance(metrics, dict):
            for name in sorted(metrics.keys()):
                metric = metrics[name]
                if not isinstance(metric, (Metric, MetricCollection)):
                    raise ValueError(
                        f"Value {metric} belonging to key {name} is not an instance of"
                        " `torchmetrics.Metric` or `torchmetrics.MetricCollection`"
                    )
                if isinstance(metric, Metric):
                    self[name] = metric
                else:
                    _absorb(name, metric)
        elif isinstance(metrics, Sequence):
            for metric in metrics:
                if not isinstance(metric, (Metric, MetricCollection)):
                    raise ValueError(
                        f"Input {metric} to `MetricCollection` is not a instance of"
                        " `torchmetrics.Metric` or `torchmetrics.MetricCollection`"
                    )
                if isinstance(metric, Metric):
                    name = metric.__class__.__name__
                    if name in self:
                        raise ValueError(f"Encountered two metrics both named {name}")
                    self[name] = metric
                else:
                    _absorb(None, metric)
        else:
            raise ValueError(
                "Unknown input to MetricCollection. Expected, `Metric`, `MetricCollection` or `dict`/`sequence` of the"
                f" previous, but got {metrics}"
            )
        self._groups_checked = False
        if self._enable_compute_groups:
            self._init_compute_groups()
        else:
            self._groups = {}

    def _init_compute_groups(self) -> None:
        if isinstance(self._enable_compute_groups, list):
            self._groups = dict(enumerate(self._enable_compute_groups))
            for v in self._groups.values():
                for metric in v:
                    if metric not in self:
                        raise ValueError(
                            f"Input {metric} in `compute_groups` argument does not match a metric in the collection."
                            f" Please make sure that {self._enable_compute_groups} matches {self.keys(keep_base=True)}"
                        )
            self._groups_checked = True
        else:
            self._groups = {i: [str(k)] for i, k in enumerate(self.keys(keep_base=True))}

    @property
    def compute_groups(self) -> Dict[int, List[str]]:
        return self._groups

    def _set_name(self, base: str) -> str:
        name = base if self.prefix is None else self.prefix + base
        return name if self.postfix is None else name + self.postfix

    def _to_renamed_ordered_dict(self) -> OrderedDict:
        od = OrderedDict()
        for k, v in self._modules.items():
            od[self._set_name(k)] = v
        return od

    def __iter__(self) -> Iterator[Hashable]:
        return iter(self.keys())

    def keys(self, keep_base: bool = False) -> Iterable[Hashable]:  # type: ignore[override]
        if keep_base:
            return self._modules.keys()
        return self._to_renamed_ordered_dict().keys()

    def items(self, keep_base: bool = False, copy_state: bool = True) -> Iterable[Tuple[str, Metric]]:  # type: ignore
        self._compute_groups_create_state_ref(copy_state)
        if keep_base:
            return self._modules.items()
        return self._to_renamed_ordered_dict().items()

    def values(self, copy_state: bool = True) -> Iterable[Metric]:  # type: ignore[override]
        self._compute_groups_create_state_ref(copy_state)
        return self._modules.values()

    def __getitem__(self, key: str, copy_state: bool = True) -> Metric:  # type: ignore[override]
        self._compute_groups_create_state_ref(copy_state)
        return self._modules[key]

    @staticmethod
    def _check_arg(arg: Optional[str], name: str) -> Optional[str]:
        if arg is None or isinstance(arg, str):
            return arg
        raise ValueError(f"Expected input `{name}` to be a string, but got {type(arg)}")

    def __repr__(self) -> str:
        out = super().__repr__()[:-2]
        if self.prefix:
            out += f",\n  prefix={self.prefix}{',' if self.postfix else ''}"
        if self.postfix:
            out += f"{',' if not self.prefix else ''}\n  postfix={self.postfix}"
        return out + "\n)"

    def set_dtype(self, dst_type: Union[str, torch.dtype]) -> "MetricCollection":
        for m in self.values(copy_state=False):
            m.set_dtype(dst_type)
        return self

    def plot(
        self,
        val: Optional[Union[Dict, Sequence[Dict]]] = None,
        ax: Optional[Union[_AX_TYPE, Sequence[_AX_TYPE]]] = None,
        together: bool = False,
    ) -> Sequence[_PLOT_OUT_TYPE]:
        if not isinstance(together, bool):
            raise ValueError(f"Expected argument `together` to be a boolean, but got {type(together)}")
        if ax is not None and not together and not (isinstance(ax, Sequence) and len(ax) == len(self)):
            raise ValueError(
                "Expected argument `ax` to be a sequence of matplotlib axis objects with the same length as the "
                f"number of metrics in the collection, but got {type(ax)} when `together=False`"
            )
        val = val or self.compute()
        if together:
            return plot_single_or_multi_val(val, ax=ax)
        out = []
        for i, (k, m) in enumerate(self.items(keep_base=True, copy_state=False)):
            if isinstance(val, dict):
                f, a = m.plot(val[k], ax=ax[i] if ax is not None else ax)
            else:
                f, a = m.plot([v[k] for v in val], ax=ax[i] if ax is not None else ax)
            out.append((f, a))
        return out
