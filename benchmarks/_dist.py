"""Shared plumbing of the multi-rank benchmarks (one process per GPU under ``torch.distributed.run``; gloo on CPU).

``setup()`` reads RANK / LOCAL_RANK / WORLD_SIZE, pins the device and initialises the process group (RCCL = backend
"nccl" on ROCm); ``barrier_sync`` brackets timed regions (barrier + device synchronize); ``max_over_ranks`` reports
the slowest rank, as the driver's contract asks for bench.py."""
import os
from typing import Any, Dict, Tuple

import torch
import torch.distributed as dist


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
