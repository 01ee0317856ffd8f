"""torchrun environment contract.

``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT`` are read exactly as
the reference scripts do (``Fine-Tuning/qwen3-8b-qlora-dist.py:15-16``,
``LLM_Distributed_Trainning/PyTorch/ddp_basics/ddp_gpt_wikitext2.py:170-182``); a missing
``WORLD_SIZE`` means single-process.
"""
from __future__ import annotations

import dataclasses
import os


@dataclasses.dataclass(frozen=True)
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    local_world_size: int = 1
    master_addr: str = "127.0.0.1"
    master_port: int = 29500

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def dist_env() -> DistEnv:
    e = os.environ
    world = int(e.get("WORLD_SIZE", 1))
    return DistEnv(
        rank=int(e.get("RANK", 0)),
        local_rank=int(e.get("LOCAL_RANK", 0)),
        world_size=world,
        local_world_size=int(e.get("LOCAL_WORLD_SIZE", world)),
        master_addr=e.get("MASTER_ADDR", "127.0.0.1"),
        master_port=int(e.get("MASTER_PORT", 29500)),
    )
