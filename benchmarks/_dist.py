"""Shared plumbing of the multi-rank benchmarks (one process per GPU; RCCL = backend "nccl" on ROCm, gloo on CPU).

``launch(gpus, script)`` makes ``--gpus N`` mean N ranks: called first thing in ``main()`` (before any GPU call), it

* returns at once when the process already runs under a launcher (``WORLD_SIZE`` set) whose world size equals N,
* exits non-zero when ``WORLD_SIZE`` disagrees with ``--gpus`` (a scaling run must never silently run the wrong N),
* otherwise, for N > 1, starts ``torch.distributed.run --nproc-per-node N`` on 127.0.0.1 as a CHILD process with the
  same script and arguments and exits with its return code (no exec: the parent has not touched the GPU, and the
  children initialise it themselves).

``setup()`` reads RANK / LOCAL_RANK / WORLD_SIZE, pins the device and initialises the process group;
``barrier_sync`` brackets timed regions (barrier + device synchronize); ``max_over_ranks`` reports the slowest rank,
as the driver's contract asks for bench.py.  Reference sync being timed: ``S/utilities/distributed.py:97-147``."""
import os
import socket
import subprocess
import sys
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(gpus: int, script: str, argv: Optional[List[str]] = None) -> None:
    """Run ``script`` on ``gpus`` ranks (see the module docstring).  Returns only in a process that is one of the
    ``gpus`` ranks (or the single rank for ``gpus == 1``)."""
    if gpus < 1:
        sys.exit(f"--gpus must be >= 1, got {gpus}")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != gpus:
            sys.exit(f"WORLD_SIZE={env_world} from the launcher disagrees with --gpus {gpus}; refusing to run a "
                     f"benchmark whose rank count differs from the one it would report")
        return
    if gpus == 1:
        return
    # device_count() does not initialise the GPU runtime on this image (is_available() would)
    ndev = torch.cuda.device_count()
    if ndev and ndev < gpus:
        sys.exit(f"--gpus {gpus} asks for more ranks than the {ndev} visible GPUs")
    argv = sys.argv[1:] if argv is None else argv
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(script), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    sys.stdout.flush()
    sys.exit(subprocess.call(cmd, env=env))


def setup() -> Tuple[int, int, torch.device]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo", rank=rank, world_size=world)
    return world, rank, device


def sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize()


def barrier_sync(device: torch.device, world: int) -> None:
    if world > 1:
        dist.barrier()
    sync(device)


def max_over_ranks(x: float, device: torch.device, world: int) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def dist_info(world: int) -> Dict[str, Any]:
    from torchmetrics_amd.parallel.sync import comm_stats

    return {"world_size_seen": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None, "engine_collectives": comm_stats()}


def teardown(world: int) -> None:
    if world > 1 and dist.is_initialized():
        dist.destroy_process_group()
