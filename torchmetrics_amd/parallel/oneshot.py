"""One-shot intra-node all-reduce over xGMI peer reads (``csrc/comm/oneshot_allreduce.hip``).

Used by the sync engine (:mod:`torchmetrics_amd.parallel.sync`) for reduce buckets of at most ``slot_bytes``
(256 KiB by default) when the process group runs on RCCL and every rank of it lives on this node.  Per call: one
kernel per rank, no host round trip.  Every rank publishes its bucket in a buffer the peers have mapped, raises a
flag in each peer's flag array and reduces the W copies straight out of the peers' HBM (rank order, so every rank
gets bit-identical sums).  Larger buckets (FID's 32 MiB covariances) stay on RCCL's ring, which is per-link
bandwidth-bound; the one-shot path is latency-bound and wins below a few hundred KiB.

The reference has no counterpart (it gathers each state with ``barrier`` + 2 ``all_gather``,
``S/utilities/distributed.py:97-147``); SURVEY.md §2.2 / §7.1.5 asks for this path.

Setup (once per process group): every rank ``hipMalloc``s one buffer, exports it with ``hipIpcGetMemHandle`` and the
handles are exchanged with ``all_gather_object``; peers open them with ``hipIpcOpenMemHandle``.  Setup also checks
that all ranks are on one host and on distinct devices; otherwise the path is disabled for that group.

Failure semantics (never a silent partial result):

* a peer wait blocks up to ``timeout_s``: ``TORCHMETRICS_AMD_ONESHOT_TIMEOUT_S`` if set, else the process group's own
  timeout (the time RCCL itself would wait), so a rank that reaches ``compute()`` seconds after its peers (rank 0
  checkpointing or logging) simply gets the right sums;
* on a timeout the kernel reduces nothing, disowns the call on every rank (two-phase protocol in the ``.hip`` file)
  and ORs ``ONESHOT_FAILED`` into the status word the caller passed -- the metric's deferred-validation word, which
  ``compute()`` reads once anyway -- so EVERY rank raises ``RuntimeError`` before a value is returned;
* raising that error disables every communicator of the process (:func:`disable_all`): all ranks raised, so all
  ranks take the RCCL path from the next sync on and their collective sequences stay matched.
"""
import os
import socket
import threading
import weakref
from datetime import timedelta
from typing import Any, Dict, Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

_OPS = {"sum": 0, "mean": 0, "max": 1, "min": 2}
_DTYPES = (torch.float32, torch.float64, torch.int64, torch.int32)
DEFAULT_SLOT_BYTES = 256 * 1024


def _enabled_by_env() -> bool:
    """Opt-in (``TORCHMETRICS_AMD_ONESHOT=1``): the path has run on one device with two processes, never across
    distinct GPUs over xGMI, so the engine keeps RCCL for every bucket unless asked (a coherence or protocol issue on
    a real xGMI mesh would otherwise show up as a long in-kernel wait on every multi-GPU sync)."""
    return os.environ.get("TORCHMETRICS_AMD_ONESHOT", "0") not in ("0", "false", "False", "")


def _resolve_group(group: Optional[Any]) -> Any:
    return group if group is not None else dist.distributed_c10d._get_default_group()


def group_timeout_s(group: Optional[Any] = None) -> float:
    """How long a peer wait may block: ``TORCHMETRICS_AMD_ONESHOT_TIMEOUT_S``, else the group's own timeout (what RCCL
    would wait before its watchdog fires), else torch's default for the backend."""
    env = os.environ.get("TORCHMETRICS_AMD_ONESHOT_TIMEOUT_S")
    if env:
        return float(env)
    g = _resolve_group(group)
    backend = dist.get_backend(g)
    dev = torch.device("cuda") if backend == "nccl" else torch.device("cpu")
    try:
        t = g._get_backend(dev).options._timeout
        if isinstance(t, timedelta) and t.total_seconds() > 0:
            return t.total_seconds()
    except Exception:  # noqa: BLE001 - private API, fall back to the documented default
        pass
    try:
        return dist.distributed_c10d._get_default_timeout(backend).total_seconds()
    except Exception:  # noqa: BLE001
        return 600.0


class OneShotAllReduce:
    """Peer-mapped buffers of one process group plus the call counter (``epoch``) that pairs the ranks' flags.

    Args:
        group: the process group (``None`` = WORLD).
        slot_bytes: the largest bucket this communicator reduces.
        allow_shared_device: permit several ranks on one device (test harness only; RCCL itself refuses it).
    """

    def __init__(self, group: Optional[Any] = None, slot_bytes: int = DEFAULT_SLOT_BYTES,
                 allow_shared_device: bool = False) -> None:
        from torchmetrics_amd import ops

        self._ops = ops._ops()
        self.group = group
        self.slot_bytes = int(slot_bytes)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device("cuda", torch.cuda.current_device())
        dev = self.device.index
        # a local failure (allocation / export) must not skip the setup collectives: every rank reaches the
        # all_gather_object and the agreement all_reduce below, and a failed rank turns the path off for all
        self._own = 0
        handle = None
        try:
            self._own = int(self._ops.ipc_buffer_alloc(int(self._ops.oneshot_buffer_bytes(self.slot_bytes)), dev))
            handle = self._ops.ipc_get_handle(self._own, dev).tolist()
        except RuntimeError:
            handle = None
        info = (socket.gethostname(), dev, os.getpid(), handle)
        infos: list = [None] * self.world
        dist.all_gather_object(infos, info, group=group)
        same_host = all(i[0] == infos[0][0] for i in infos)
        distinct = len({i[1] for i in infos}) == self.world
        exported = all(i[3] is not None for i in infos)
        self.usable = bool(same_host and exported and (distinct or allow_shared_device) and self.world <= 16)
        self._opened = []
        ptrs = []
        ok = self.usable
        if ok:
            try:
                for r, i in enumerate(infos):
                    if r == self.rank:
                        ptrs.append(self._own)
                    else:
                        p = int(self._ops.ipc_open_handle(torch.tensor(i[3], dtype=torch.uint8), dev))
                        self._opened.append(p)
                        ptrs.append(p)
            except RuntimeError:
                ok = False
        # every rank must take the same path: agree on the outcome (MIN over ranks)
        flag_dev = self.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
        agree = torch.tensor([1 if ok else 0], dtype=torch.int32, device=flag_dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MIN, group=group)
        self.usable = bool(int(agree.item()))
        self._peers = torch.tensor(ptrs or [self._own], dtype=torch.int64)
        self._status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.timeout_s = group_timeout_s(group)
        self.epoch = 0
        self.calls = 0
        self.failed = False
        _instances.add(self)

    def supports(self, buf: Tensor) -> bool:
        return (
            self.usable
            and buf.device == self.device
            and buf.dtype in _DTYPES
            and buf.numel() * buf.element_size() <= self.slot_bytes
            and not torch.cuda.is_current_stream_capturing()  # the epoch is a launch argument
        )

    def all_reduce(self, buf: Tensor, op: str = "sum", err: Optional[Tensor] = None) -> Tensor:
        """In-place reduction of a contiguous 1-D ``buf`` across the group (``mean`` is left as a sum).

        ``err``: an int32 device word that receives ``ONESHOT_FAILED`` if the call fails; the caller MUST read it (or
        call :meth:`check`) before using ``buf``.  Without ``err`` the status is checked here (one device sync)."""
        if not self.usable:
            raise RuntimeError("one-shot all-reduce: communicator is disabled")
        self.epoch += 1
        if self.epoch >= 2**31 - 1:
            raise RuntimeError("one-shot all-reduce: epoch counter exhausted")
        inp = buf.contiguous()
        self._ops.oneshot_allreduce(inp, buf, self._peers, self.rank, self.slot_bytes, self.epoch, _OPS[op], True,
                                    float(self.timeout_s), self._status, err)
        self.calls += 1
        if err is None:
            self.check()
        return buf

    def check(self) -> None:
        """Raise (and disable every communicator) if a call ever timed out or was disowned by a peer (one device
        sync)."""
        code = int(self._status.item())
        if code != 0:
            disable_all()
            raise RuntimeError(failure_message(code, self.timeout_s))

    def disable(self) -> None:
        """Stop using this communicator (after a failure every rank raised, so every rank disables it; buffers stay
        mapped until :meth:`close`, a late peer's kernel may still be reading them)."""
        self.usable = False
        self.failed = True

    def close(self) -> None:
        dev = self.device.index
        for p in self._opened:
            self._ops.ipc_close_handle(p, dev)
        self._opened = []
        if self._own:
            self._ops.ipc_buffer_free(self._own, dev)
            self._own = 0
        self.usable = False


def failure_message(code: int = 1, timeout_s: Optional[float] = None) -> str:
    what = "a peer did not arrive" if code & 1 else "a peer timed out and disowned the call"
    limit = f" within {timeout_s:g} s" if timeout_s is not None and code & 1 else ""
    return (f"one-shot all-reduce failed: {what}{limit}; the metric states were NOT synchronised and no value is "
            "returned. The one-shot path is now disabled on every rank; the next sync uses RCCL "
            "(raise the limit with TORCHMETRICS_AMD_ONESHOT_TIMEOUT_S or the process group's timeout).")


_instances: "weakref.WeakSet[OneShotAllReduce]" = weakref.WeakSet()


def disable_all() -> None:
    """Disable every communicator of this process (called on every rank when a one-shot failure is raised)."""
    for c in list(_instances):
        c.disable()


# registry: id(resolved group) -> (weakref to the group, communicator or None); the weakref guards against a new
# group allocated at a destroyed group's address (a re-initialised WORLD included)
_registry: Dict[int, Tuple[Any, Optional[OneShotAllReduce]]] = {}
_lock = threading.Lock()


def get_oneshot(group: Optional[Any] = None) -> Optional[OneShotAllReduce]:
    """The group's communicator (created collectively on first use), or ``None`` where the path does not apply.

    Every rank reaches this call at the same point of the engine's collective sequence (the decision depends only on
    the backend, the env switch and the bucket size, which agree across ranks), so the setup collective is safe.
    """
    g = _resolve_group(group)
    key = id(g)
    with _lock:
        hit = _registry.get(key)
        if hit is not None:
            if hit[0]() is g:
                comm = hit[1]
                return comm if comm is not None and comm.usable else None
            stale = _registry.pop(key)[1]  # the group this entry belonged to is gone
            if stale is not None:
                stale.close()
    comm = None
    if _enabled_by_env() and torch.cuda.is_available():
        from torchmetrics_amd import ops

        if ops.load_native(strict=False):
            comm = OneShotAllReduce(group)  # collective; ranks agree on `usable` inside
    with _lock:
        _registry[key] = (weakref.ref(g), comm)
    return comm if comm is not None and comm.usable else None


def reset_registry() -> None:
    with _lock:
        for _, c in _registry.values():
            if c is not None:
                c.close()
        _registry.clear()


__all__ = ["OneShotAllReduce", "get_oneshot", "reset_registry", "disable_all", "group_timeout_s", "DEFAULT_SLOT_BYTES"]
