"""Process groups and collectives.

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` — which IS RCCL on ROCm,
running intra-node over xGMI (8×MI355X full mesh, 7 links/GPU) — or ``gloo`` on CPU.  Same
``env://`` contract as the reference (``ddp_gpt_wikitext2.py:170-182``): a missing
``WORLD_SIZE`` means single-process, and every helper degrades to a no-op.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..runtime.env import dist_env


def local_device_index(local_rank: int) -> int:
    """GPU of this rank: ``local_rank``, or ``local_rank % device_count`` under ``LIPA_SHARE_GPU=1``
    (a multi-rank rehearsal of the distributed path on a box with fewer GPUs than ranks; pair it with
    ``LIPA_DIST_BACKEND=gloo``, since RCCL refuses two ranks on one device)."""
    if os.environ.get("LIPA_SHARE_GPU", "0") == "1" and torch.cuda.is_available():
        return local_rank % max(1, torch.cuda.device_count())
    return local_rank


def init_distributed(backend: str | None = None, timeout_s: int = 1800) -> tuple[int, int, int]:
    """Initialise the default group from torchrun env vars.  Returns (rank, local_rank, world).
    ``LIPA_DIST_BACKEND`` overrides the backend (default: nccl = RCCL with GPUs, else gloo)."""
    env = dist_env()
    dev = local_device_index(env.local_rank)
    if env.world_size > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("LIPA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(dev)
        kw = dict(backend=backend, init_method="env://", timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", dev)
        try:
            dist.init_process_group(**kw)
        except TypeError:
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(dev)
    return env.rank, env.local_rank, env.world_size


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def is_main() -> bool:
    return rank() == 0


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    if is_dist():
        if dist.get_backend(group) == "nccl" and hasattr(dist.ReduceOp, "AVG"):
            dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(t, group=group)
            t.div_(dist.get_world_size(group))
    return t


def all_reduce_max(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
