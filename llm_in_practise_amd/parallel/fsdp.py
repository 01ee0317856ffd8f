"""FSDP-style API over the ZeRO engine (C2 ``fsdp_gpt_wikitext2.py:271-316``,
C3 ``fsdp2_gpt_wikitext2.py:261-293``).

One sharded-parameter runtime serves both vocabularies: ``ShardingStrategy.FULL_SHARD`` = ZeRO-3
(per wrapped block all-gather in forward/backward, reduce-scatter of gradients),
``SHARD_GRAD_OP`` = ZeRO-2, ``NO_SHARD`` = replicated (DDP semantics).  ``MixedPrecision(bf16)``
maps to bf16 compute with fp32 master shards; ``CPUOffload(offload_params=True)`` to the host
optimizer.  ``transformer_auto_wrap_policy({Block})`` selects the partition units (the default
is every element of every ``nn.ModuleList``); FSDP2's ``fully_shard(model)`` at the root only
(what C3 does) shards the whole model as one unit list.  ``get_state_dict(full_state_dict=True)``
gathers the consolidated state dict (collective) for a rank-0 save.
"""
from __future__ import annotations

import enum
import functools

import torch
import torch.nn as nn

from .zero import ZeroEngine


class ShardingStrategy(enum.Enum):
    FULL_SHARD = 3
    SHARD_GRAD_OP = 2
    NO_SHARD = 0


class MixedPrecision:
    def __init__(self, param_dtype=None, reduce_dtype=None, buffer_dtype=None):
        self.param_dtype, self.reduce_dtype, self.buffer_dtype = param_dtype, reduce_dtype, buffer_dtype


class CPUOffload:
    def __init__(self, offload_params: bool = False):
        self.offload_params = offload_params


def transformer_auto_wrap_policy(transformer_layer_cls: set | tuple):
    cls = tuple(transformer_layer_cls)
    return functools.partial(_wrap_by_class, cls=cls)


def _wrap_by_class(module: nn.Module, cls=()):
    return [m for m in module.modules() if isinstance(m, cls)]


class FullyShardedDataParallel(nn.Module):
    """``FSDP(model, auto_wrap_policy=..., sharding_strategy=..., mixed_precision=..., cpu_offload=...)``.

    Training loop surface: ``loss = fsdp(x, y)``; ``fsdp.backward(loss)`` (or ``loss.backward()``
    followed by ``fsdp.step()``) — the optimizer lives in the engine (``fsdp.optimizer``)."""

    def __init__(self, module: nn.Module, auto_wrap_policy=None, sharding_strategy=ShardingStrategy.FULL_SHARD,
                 mixed_precision: MixedPrecision | None = None, cpu_offload: CPUOffload | None = None,
                 sync_module_states: bool = True, device_id=None, lr: float = 3e-4, weight_decay: float = 0.0,
                 grad_clip: float = 0.0, **_):
        super().__init__()
        cfg = {"zero_optimization": {"stage": sharding_strategy.value, "stage3_param_persistence_threshold": 0},
               "gradient_clipping": grad_clip,
               "optimizer": {"type": "AdamW", "params": {"lr": lr, "weight_decay": weight_decay}}}
        if mixed_precision is not None and mixed_precision.param_dtype == torch.bfloat16:
            cfg["bf16"] = {"enabled": True}
        if cpu_offload is not None and cpu_offload.offload_params:
            cfg["zero_optimization"]["offload_optimizer"] = {"device": "cpu"}
        units = auto_wrap_policy(module) if auto_wrap_policy is not None else None
        self.engine = ZeroEngine(module, cfg, lr=lr, weight_decay=weight_decay, units=units)
        self.module = module

    @property
    def optimizer(self):
        return self.engine

    def forward(self, *a, **kw):
        return self.engine(*a, **kw)

    def backward(self, loss):
        self.engine.backward(loss)

    def step(self):
        self.engine.step()

    def zero_grad(self):
        self.engine.zero_grad()

    def full_state_dict(self) -> dict:
        return self.engine.consolidated_state_dict()


FSDP = FullyShardedDataParallel


def fully_shard(model: nn.Module, mesh=None, reshard_after_forward: bool = True, mp_policy=None,
                offload_policy=None, **kw) -> FullyShardedDataParallel:
    """FSDP2 entry point (root-level sharding, ``fsdp2_gpt_wikitext2.py:286``)."""
    mp = MixedPrecision(param_dtype=getattr(mp_policy, "param_dtype", None)) if mp_policy is not None else None
    strategy = ShardingStrategy.FULL_SHARD if reshard_after_forward else ShardingStrategy.SHARD_GRAD_OP
    return FullyShardedDataParallel(model, None, strategy, mp, **kw)


def get_state_dict(model, optimizers=None, options=None) -> tuple[dict, dict]:
    """``torch.distributed.checkpoint.state_dict.get_state_dict`` analogue with
    ``StateDictOptions(full_state_dict=True)``: consolidated model state (collective on every
    rank) and the rank-local optimizer shard."""
    eng = model.engine if isinstance(model, FullyShardedDataParallel) else model
    msd = eng.consolidated_state_dict()
    osd = {"exp_avg": eng.exp_avg.detach().cpu(), "exp_avg_sq": eng.exp_avg_sq.detach().cpu(),
           "step": eng.opt_step}
    return msd, osd
