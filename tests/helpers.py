"""Test harness modelled on the reference ``MetricTester`` (``T/helpers/testers.py:74-474``).

* ``run_class_test``: per-batch ``forward`` vs oracle on the batch, final ``compute`` vs oracle on all data,
  plus pickling, clone, ``hash``, empty default ``state_dict`` and const-attribute guards.
* ``run_ddp_class_test``: the same on a 2-rank gloo pool (rank-strided batches; final value vs oracle on all data).
* ``run_functional_test``: functional vs oracle per batch.
"""
import os
import pickle
import socket
import sys
from functools import partial
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

NUM_PROCESSES = 2


def _to_np(x: Any) -> Any:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().double().numpy()
    if isinstance(x, dict):
        return {k: _to_np(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_np(v) for v in x]
    return x


def assert_close(ours: Any, ref: Any, atol: float = 1e-6, rtol: float = 1e-5) -> None:
    if isinstance(ref, dict):
        for k in ref:
            assert_close(ours[k], ref[k], atol, rtol)
        return
    if isinstance(ref, (list, tuple)) and not isinstance(ours, torch.Tensor):
        assert len(ours) == len(ref)
        for a, b in zip(ours, ref):
            assert_close(a, b, atol, rtol)
        return
    np.testing.assert_allclose(_to_np(ours), _to_np(ref), atol=atol, rtol=rtol, equal_nan=True)


def _class_test_body(
    rank: int,
    world: int,
    preds: torch.Tensor,
    target: torch.Tensor,
    metric_class: Any,
    metric_args: Dict,
    ref_fn: Callable,
    atol: float,
    device: str,
    check_batch: bool,
    fragment_kwargs: Dict,
) -> None:
    metric = metric_class(**metric_args)
    for attr in ("is_differentiable", "higher_is_better", "full_state_update"):
        try:
            setattr(metric, attr, None)
            raise AssertionError(f"const attribute {attr} was writable")
        except RuntimeError:
            pass
    metric = metric.to(device)
    metric = pickle.loads(pickle.dumps(metric))
    clone = metric.clone()
    assert type(clone) is type(metric)
    num_batches = preds.shape[0]
    for i in range(rank, num_batches, world):
        p, t = preds[i].to(device), target[i].to(device)
        batch_val = metric(p, t, **fragment_kwargs)
        if check_batch and world == 1:
            assert_close(batch_val, ref_fn(preds[i], target[i]), atol=atol)
    assert isinstance(hash(metric), int)
    if not any(metric._persistent.values()):
        assert len(metric.state_dict()) == 0
    result = metric.compute()
    all_p = torch.cat([preds[i] for i in range(num_batches)])
    all_t = torch.cat([target[i] for i in range(num_batches)])
    assert_close(result, ref_fn(all_p, all_t), atol=atol)


def run_class_test(
    preds: torch.Tensor,
    target: torch.Tensor,
    metric_class: Any,
    ref_fn: Callable,
    metric_args: Optional[Dict] = None,
    atol: float = 1e-6,
    device: str = "cpu",
    check_batch: bool = True,
    **fragment_kwargs: Any,
) -> None:
    _class_test_body(0, 1, preds, target, metric_class, metric_args or {}, ref_fn, atol, device, check_batch,
                     fragment_kwargs)


def run_functional_test(
    preds: torch.Tensor,
    target: torch.Tensor,
    metric_fn: Callable,
    ref_fn: Callable,
    metric_args: Optional[Dict] = None,
    atol: float = 1e-6,
    device: str = "cpu",
) -> None:
    for i in range(preds.shape[0]):
        ours = metric_fn(preds[i].to(device), target[i].to(device), **(metric_args or {}))
        assert_close(ours, ref_fn(preds[i], target[i]), atol=atol)


# ----------------------------------------------------------------------------------------------- DDP (gloo pool)
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_entry(rank: int, world: int, port: int, fn: Callable, args: tuple, errq: Any) -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    try:
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        except RuntimeError as err:  # a port / mesh race with another test process: run_ddp retries these
            # queued once, as a rendezvous failure only (a second, traceback entry would defeat run_ddp's retry)
            errq.put(f"{_RENDEZVOUS} rank {rank}: {err!r}")
            sys.exit(3)
        fn(rank, world, *args)
    except SystemExit:
        raise  # the rendezvous failure above, already queued
    except BaseException as err:  # noqa: BLE001
        import traceback

        errq.put(f"rank {rank}: {err!r}\n{traceback.format_exc()}")
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


_RENDEZVOUS = "rendezvous failure"


def run_ddp(fn: Callable, *args: Any, world: int = NUM_PROCESSES, attempts: int = 3) -> None:
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks (spawned processes); re-raise the first failure.
    A failed rendezvous (a port taken by a concurrent test process between picking and binding it) is retried on a
    fresh port."""
    ctx = mp.get_context("spawn")
    for attempt in range(attempts):
        errq = ctx.SimpleQueue()
        port = _free_port()
        procs = [ctx.Process(target=_ddp_entry, args=(r, world, port, fn, args, errq)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
        for p in procs:
            if p.is_alive():
                p.kill()
        errors = []
        while not errq.empty():
            errors.append(errq.get())
        if errors and all(e.startswith(_RENDEZVOUS) for e in errors) and attempt + 1 < attempts:
            continue
        if errors:
            real = [e for e in errors if not e.startswith(_RENDEZVOUS)]
            raise AssertionError((real or errors)[0])
        for p in procs:
            assert p.exitcode == 0, f"ddp worker exited with {p.exitcode}"
        return


def run_ddp_class_test(
    preds: torch.Tensor,
    target: torch.Tensor,
    metric_class: Any,
    ref_fn: Callable,
    metric_args: Optional[Dict] = None,
    atol: float = 1e-6,
) -> None:
    run_ddp(_class_test_body, preds, target, metric_class, metric_args or {}, ref_fn, atol, "cpu", False, {})
