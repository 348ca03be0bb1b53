"""Packed state arenas: the reducible tensor states of a metric (or of every compute-group leader of a collection)
live as contiguous views of ONE flat buffer per (reduction, dtype, device).

Reference: every state is its own tensor and is synced on its own (``S/metric.py:195-272`` registers them,
``S/metric.py:427-457`` gathers them one by one).  Here the sync engine (:mod:`torchmetrics_amd.parallel.sync`) finds
the bucket of a (reduction, dtype, device) already laid out back to back and sends it as one span: one ``clone`` of the
arena (the local states are never touched by the collective) instead of a ``torch.cat`` of its members on every sync.

The layout is an invariant the engine *checks* (``contiguous_span``), never assumes: a state that an update, ``reset()``
or ``load_state_dict`` rebinds to a fresh tensor simply falls out of the span, the next sync re-packs (one ``cat`` into
a new buffer, the states rebound to views of it), and a metric that keeps rebinding its states is left unpacked after a
few attempts (its buckets go through the ``cat`` path, exactly as without an arena).  Packing never changes a state's
value, shape or dtype -- only where it lives -- so ``state_dict`` keys and values are unchanged.
"""
from typing import Dict, List, Optional, Sequence, Tuple

import torch
from torch import Tensor

# re-packs of one metric's states after its first packing before it is left unpacked (its update rebinds states)
MAX_REPACKS = 3

_Key = Tuple[str, torch.dtype, torch.device]


def _reduce_kind(fn) -> Optional[str]:
    global _KINDS
    if _KINDS is None:  # (imported lazily: utilities.data imports this package)
        from torchmetrics_amd.utilities.data import dim_zero_max, dim_zero_mean, dim_zero_min, dim_zero_sum

        _KINDS = {dim_zero_sum: "sum", dim_zero_mean: "mean", dim_zero_max: "max", dim_zero_min: "min"}
    return _KINDS.get(fn) if fn is not None and not isinstance(fn, str) else None


_KINDS: Optional[dict] = None


def contiguous_span(tensors: Sequence[Tensor]) -> Optional[Tensor]:
    """A 1-D view covering ``tensors`` when they lie back to back, in this order, in one storage; else ``None``."""
    first = tensors[0]
    es = first.element_size()
    base = first.data_ptr()
    nxt = base
    dt = first.dtype
    for t in tensors:
        if t.data_ptr() != nxt or t.dtype != dt or not t.is_contiguous():
            return None
        nxt += t.numel() * es
    # adjacent addresses may still be two allocations side by side in one allocator segment: the first and the last
    # tensor must share a storage (separate storages never overlap, so the ones in between share it too)
    last = tensors[-1]
    if last is not first and last.untyped_storage().data_ptr() != first.untyped_storage().data_ptr():
        return None
    return torch.as_strided(first, ((nxt - base) // es,), (1,))


def _packable(t) -> bool:
    return isinstance(t, Tensor) and t.layout == torch.strided and not t.requires_grad and not t.is_sparse


def buckets_of(metrics: Sequence) -> Dict[_Key, List[Tuple[object, str, Tensor]]]:
    """Reducible tensor states of ``metrics`` per (reduction, dtype, device), in the sync engine's order."""
    out: Dict[_Key, List[Tuple[object, str, Tensor]]] = {}
    for m in metrics:
        d = m.__dict__
        for name, fn in m._reductions.items():
            t = d.get(name)
            kind = _reduce_kind(fn)
            if kind is None or not _packable(t):
                continue
            out.setdefault((kind, t.dtype, t.device), []).append((m, name, t))
    return out


def is_packed(metrics: Sequence) -> bool:
    return all(len(items) < 2 or contiguous_span([t for _, _, t in items]) is not None
               for items in buckets_of(metrics).values())


def pack_items(items: Sequence[Tuple[object, str, Tensor]]) -> Optional[Tensor]:
    """Pack one bucket given as distinct ``(metric, attr, tensor)`` states (a state shared by several metrics -- a
    compute group -- appears once; the caller re-points the sharers).  Returns the bucket's span."""
    ts = [t for _, _, t in items]
    span = contiguous_span(ts)
    if span is not None:
        return span
    buf = torch.cat([t.reshape(-1) for t in ts])
    off = 0
    for m, name, t in items:
        n = t.numel()
        m.__dict__[name] = buf[off:off + n].view(t.shape)
        off += n
    return buf


def pack(metrics: Sequence, force: bool = False) -> bool:
    """Lay the reducible states of ``metrics`` out as views of one buffer per bucket (one ``cat`` per bucket that is
    not laid out yet).  Metrics that have been re-packed ``MAX_REPACKS`` times are skipped unless ``force``.
    Returns True if every bucket is now one span."""
    live = [m for m in metrics if force or m.__dict__.get("_arena_repacks", 0) <= MAX_REPACKS]
    touched = set()
    for items in buckets_of(live).values():
        ts = [t for _, _, t in items]
        if len(ts) < 2 or contiguous_span(ts) is not None:
            continue
        buf = torch.cat([t.reshape(-1) for t in ts])
        off = 0
        for m, name, t in items:
            n = t.numel()
            m.__dict__[name] = buf[off:off + n].view(t.shape)
            off += n
            touched.add(id(m))
    for m in live:
        if id(m) in touched:
            d = m.__dict__
            d["_arena_repacks"] = d.get("_arena_repacks", -1) + 1
    return len(live) == len(metrics) and is_packed(metrics)
