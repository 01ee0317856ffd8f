"""Device selection and HBM accounting.

Reference behaviour: every script picks ``cuda`` if available else ``cpu``
(``llm-demo/minigpt/train.py:7``) and distributed scripts call
``torch.cuda.set_device(local_rank)`` before building the model
(``Fine-Tuning/qwen3-8b-lora-dist.py:25``).  On ROCm the ``cuda`` device *is* the
HIP device; we keep the name so user code stays unchanged.
"""
from __future__ import annotations

import functools
import os

import torch


def get_device(local_rank: int | None = None) -> torch.device:
    """Return the compute device for this process, binding the HIP device first."""
    if torch.cuda.is_available():
        if local_rank is None:
            local_rank = int(os.environ.get("LOCAL_RANK", 0))
        torch.cuda.set_device(local_rank)
        return torch.device("cuda", local_rank)
    return torch.device("cpu")


@functools.lru_cache(maxsize=None)
def is_gfx950(index: int = 0) -> bool:
    if not torch.cuda.is_available():
        return False
    props = torch.cuda.get_device_properties(index)
    return "gfx950" in getattr(props, "gcnArchName", "")


def synchronize() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def hbm_stats(device: torch.device | None = None) -> dict:
    """Allocated / reserved / peak HBM in GiB (288 GB per MI355X)."""
    if not torch.cuda.is_available():
        return {}
    g = 1024 ** 3
    free, total = torch.cuda.mem_get_info(device)
    return {
        "allocated_gib": torch.cuda.memory_allocated(device) / g,
        "reserved_gib": torch.cuda.memory_reserved(device) / g,
        "peak_gib": torch.cuda.max_memory_allocated(device) / g,
        "free_gib": free / g,
        "total_gib": total / g,
    }
