"""DeepSpeed-JSON config semantics without DeepSpeed.

Accepts the reference configs verbatim (``Fine-Tuning/ds_zero3_config.json``,
``LLM_Distributed_Trainning/DeepSpeed/*/ds_config.json``) and resolves ``"auto"`` the way the
HF integration does [ext]:
  * ``train_micro_batch_size_per_gpu``  ← per-device batch size
  * ``gradient_accumulation_steps``     ← trainer GA
  * ``train_batch_size``                ← micro × GA × world
  * ``reduce_bucket_size``              ← hidden²
  * ``stage3_prefetch_bucket_size``     ← 0.9 · hidden²
  * ``stage3_param_persistence_threshold`` ← 10 · hidden
and checks ``train_batch_size == micro × GA × world``.  Precedence between a client optimizer
and a config ``optimizer`` block is explicit: the config block wins when present
(``config_optimizer_wins``), matching DeepSpeed's behaviour when both are given [ext].
"""
from __future__ import annotations

import dataclasses
import json
import os


def _num(v, default=None):
    if v is None or v == "auto":
        return default
    return int(float(v)) if isinstance(v, (int, float, str)) else v


@dataclasses.dataclass
class ZeroConfig:
    stage: int = 0
    overlap_comm: bool = False
    contiguous_gradients: bool = True
    reduce_scatter: bool = True
    reduce_bucket_size: int = int(5e8)
    allgather_bucket_size: int = int(5e8)
    allgather_partitions: bool = True
    sub_group_size: int = int(1e9)
    stage3_prefetch_bucket_size: int = int(5e7)
    stage3_param_persistence_threshold: int = int(1e5)
    stage3_max_live_parameters: int = int(1e9)
    stage3_max_reuse_distance: int = int(1e9)
    stage3_gather_16bit_weights_on_model_save: bool = False
    stage3_partition_frozen_quant: bool = False     # extension: shard frozen NF4 bases too (zero.py)
    offload_optimizer: str = "none"          # "none" | "cpu"
    offload_param: str = "none"
    pin_memory: bool = False


@dataclasses.dataclass
class DSConfig:
    train_batch_size: int | None = None
    train_micro_batch_size_per_gpu: int | None = None
    gradient_accumulation_steps: int = 1
    gradient_clipping: float = 0.0
    steps_per_print: int = 10
    wall_clock_breakdown: bool = False
    bf16: bool = False
    fp16: bool = False
    fp16_loss_scale: float = 0.0             # 0 = dynamic
    fp16_initial_scale_power: int = 16
    fp16_loss_scale_window: int = 1000
    fp16_hysteresis: int = 2
    fp16_min_loss_scale: float = 1.0
    optimizer: dict | None = None            # {"type": "AdamW", "params": {...}}
    scheduler: dict | None = None            # {"type": "WarmupLR", "params": {...}}
    zero: ZeroConfig = dataclasses.field(default_factory=ZeroConfig)
    raw: dict = dataclasses.field(default_factory=dict)

    @property
    def zero_stage(self) -> int:
        return self.zero.stage

    def to_dict(self) -> dict:
        return dict(self.raw)


def load_ds_config(cfg, world_size: int = 1, micro_batch: int | None = None, grad_accum: int | None = None,
                   hidden_size: int | None = None) -> DSConfig:
    """Parse a ds_config (path, JSON string or dict) and resolve ``"auto"`` values."""
    if isinstance(cfg, DSConfig):
        return cfg
    if isinstance(cfg, str):
        if os.path.exists(cfg):
            with open(cfg) as f:
                raw = json.load(f)
        else:
            raw = json.loads(cfg)
    else:
        raw = dict(cfg or {})
    z = raw.get("zero_optimization", {}) or {}
    h2 = hidden_size * hidden_size if hidden_size else None
    zc = ZeroConfig(
        stage=int(z.get("stage", 0)),
        # DeepSpeed's default: overlapped for stage 3, not for stages 1-2
        overlap_comm=bool(z.get("overlap_comm", int(z.get("stage", 0)) == 3)),
        contiguous_gradients=bool(z.get("contiguous_gradients", True)),
        reduce_scatter=bool(z.get("reduce_scatter", True)),
        reduce_bucket_size=_num(z.get("reduce_bucket_size"), h2 or int(5e8)),
        allgather_bucket_size=_num(z.get("allgather_bucket_size"), int(5e8)),
        allgather_partitions=bool(z.get("allgather_partitions", True)),
        sub_group_size=_num(z.get("sub_group_size"), int(1e9)),
        stage3_prefetch_bucket_size=_num(z.get("stage3_prefetch_bucket_size"),
                                         int(0.9 * h2) if h2 else int(5e7)),
        stage3_param_persistence_threshold=_num(z.get("stage3_param_persistence_threshold"),
                                                10 * hidden_size if hidden_size else int(1e5)),
        stage3_max_live_parameters=_num(z.get("stage3_max_live_parameters"), int(1e9)),
        stage3_max_reuse_distance=_num(z.get("stage3_max_reuse_distance"), int(1e9)),
        stage3_gather_16bit_weights_on_model_save=bool(z.get("stage3_gather_16bit_weights_on_model_save", False)),
        stage3_partition_frozen_quant=bool(z.get("stage3_partition_frozen_quant", False)),
        offload_optimizer=(z.get("offload_optimizer") or {}).get("device", "none"),
        offload_param=(z.get("offload_param") or {}).get("device", "none"),
        pin_memory=bool((z.get("offload_optimizer") or {}).get("pin_memory", False)),
    )
    fp16 = raw.get("fp16", {}) or {}
    bf16 = raw.get("bf16", {}) or {}
    ga = _num(raw.get("gradient_accumulation_steps"), grad_accum or 1)
    if grad_accum is not None and raw.get("gradient_accumulation_steps") not in (None, "auto") and ga != grad_accum:
        raise ValueError(f"ds_config gradient_accumulation_steps={ga} != trainer grad accum {grad_accum}")
    micro = _num(raw.get("train_micro_batch_size_per_gpu"), micro_batch)
    tbs = _num(raw.get("train_batch_size"), None)
    if micro is None and tbs is not None:
        micro = tbs // (ga * world_size)
    if tbs is None and micro is not None:
        tbs = micro * ga * world_size
    if tbs is not None and micro is not None and tbs != micro * ga * world_size:
        raise ValueError(f"train_batch_size {tbs} != micro {micro} x GA {ga} x world {world_size}")
    return DSConfig(
        train_batch_size=tbs, train_micro_batch_size_per_gpu=micro, gradient_accumulation_steps=ga,
        gradient_clipping=float(raw.get("gradient_clipping", 0.0) or 0.0),
        steps_per_print=int(raw.get("steps_per_print", 10)),
        wall_clock_breakdown=bool(raw.get("wall_clock_breakdown", False)),
        bf16=bool(bf16.get("enabled", False)), fp16=bool(fp16.get("enabled", False)),
        fp16_loss_scale=float(fp16.get("loss_scale", 0) or 0),
        fp16_initial_scale_power=int(fp16.get("initial_scale_power", 16)),
        fp16_loss_scale_window=int(fp16.get("loss_scale_window", 1000)),
        fp16_hysteresis=int(fp16.get("hysteresis", 2)),
        fp16_min_loss_scale=float(fp16.get("min_loss_scale", 1)),
        optimizer=raw.get("optimizer"), scheduler=raw.get("scheduler"), zero=zc, raw=raw)
