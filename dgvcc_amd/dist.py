"""Data-parallel plumbing: frames shard over ranks; the only
exchange is one all-reduce of the flat fp32 gradient per step (RCCL over xGMI
with backend "nccl" on ROCm; gloo on CPU for tests)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend: str | None = None) -> int:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_*); returns local rank."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return local


def average_flat_(flat: torch.Tensor) -> torch.Tensor:
    """In-place mean over ranks of one flat gradient buffer (single collective)."""
    n = world()
    if n > 1:
        dist.all_reduce(flat)
        flat.div_(n)
    return flat


def broadcast_module_(module: torch.nn.Module, src: int = 0) -> None:
    """Identical initial weights/buffers on every rank."""
    if world() > 1:
        for t in module.state_dict().values():
            dist.broadcast(t, src)


def sum_moments(n_local: int):
    """Reducer for SyncSwitchWhiten2d (models/SW/ops/sync_switchwhiten.py:13-56):
    t -> (t summed over ranks, n_local * world).  Like the reference's SyncMeanCov it
    assumes every rank holds the same number of images."""
    def reduce(t: torch.Tensor):
        n = world()
        if n > 1:
            dist.all_reduce(t)
        return t, n_local * n
    return reduce
