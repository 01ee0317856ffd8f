"""Tensor parallelism for Qwen2/Qwen3 inference.

The reference serves adapters with vLLM ``--tensor-parallel-size 2`` (``Fine-Tuning/README.md:345-361``)
and otherwise runs TP=1; training never uses TP.  Here TP is a one-call transform of a loaded
model, one process per GPU (torchrun), RCCL all-reduce over xGMI:

* q / k / v / gate / up are **column-parallel**: each rank keeps a contiguous block of heads
  (``hq/tp`` query heads, ``hkv/tp`` KV heads — the GQA head→group map is preserved) or FFN
  columns; q/k norms, RoPE and flash attention run on the local heads unchanged.
* o / down are **row-parallel**: each rank multiplies its slice of the reduction dimension and
  one all-reduce per block sums the partials (the residual is added on rank 0 only, inside the
  GEMM epilogue, so the sum contains it once).  Two all-reduces of ``[tokens, hidden]`` bf16
  per layer — on an 8×MI355X xGMI mesh each is a one-hop ring over 7 links.
* LoRA follows its base: column-parallel bases shard ``lora_B`` rows (``lora_A`` replicated);
  row-parallel bases shard ``lora_A`` columns (``lora_B`` replicated) — the output all-reduce
  then sums ``Σ_r (x_r·A_rᵀ)·Bᵀ = (x·Aᵀ)·Bᵀ`` exactly.
* Embeddings, norms and the LM head stay replicated, so every rank ends with bit-identical
  logits and can sample in lockstep (SPMD decoding needs no token broadcast).
* Apply before NF4/int4 quantisation and before ``fuse_projections`` (the shards are what gets
  quantised; KV caches are sized from the rewritten local head counts in ``model.config``).

The all-reduce is wrapped in an autograd function (forward all-reduce, backward identity) so
the sharded model also back-propagates, but TP *training* (replicated-parameter gradient
sync) is out of the reference's scope and not wired into the trainers.
"""
from __future__ import annotations

import copy

import torch
import torch.distributed as dist
import torch.nn as nn


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.mark_dirty(x)
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, dy):
        return dy, None


def tp_all_reduce(x: torch.Tensor, group) -> torch.Tensor:
    """Sum row-parallel partial outputs across the TP group (in place)."""
    if group is None:
        return x
    return _ReduceFromTP.apply(x, group)


def _narrow_param(p: nn.Parameter, dim: int, start: int, n: int) -> nn.Parameter:
    return nn.Parameter(p.data.narrow(dim, start, n).clone(), requires_grad=p.requires_grad)


def _shard_linear(mod: nn.Module, dim: int, rank: int, world: int):
    """Column (dim 0: out features) or row (dim 1: in features) shard of an nn.Linear or a
    LoRA-wrapped nn.Linear, in place."""
    from ..peft.lora import LoraLayer, Linear4bit
    lora = mod if isinstance(mod, LoraLayer) else None
    lin = mod.base_layer if lora is not None else mod
    if isinstance(lin, Linear4bit):
        raise TypeError("apply_tensor_parallel: shard before NF4 quantisation (quantise the shards)")
    full = lin.weight.shape[dim]
    assert full % world == 0, f"dimension {full} not divisible by tp={world}"
    n = full // world
    lin.weight = _narrow_param(lin.weight, dim, rank * n, n)
    if dim == 0:
        lin.out_features = n
        if lin.bias is not None:
            lin.bias = _narrow_param(lin.bias, 0, rank * n, n)
    else:
        lin.in_features = n
        if lin.bias is not None and rank != 0:   # a row-parallel bias is added once (rank 0)
            lin.bias = nn.Parameter(torch.zeros_like(lin.bias), requires_grad=lin.bias.requires_grad)
    if lora is not None:
        if dim == 0:
            lora.lora_B.weight = _narrow_param(lora.lora_B.weight, 0, rank * n, n)
            lora.lora_B.out_features = n
        else:
            lora.lora_A.weight = _narrow_param(lora.lora_A.weight, 1, rank * n, n)
            lora.lora_A.in_features = n


def apply_tensor_parallel(model: nn.Module, group=None) -> nn.Module:
    """Shard a ``Qwen3ForCausalLM`` (Qwen2 or Qwen3 architecture) across ``group`` in place."""
    if group is None:
        group = dist.group.WORLD
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    from ..models.qwen3 import Qwen3ForCausalLM
    lm = next((m for m in model.modules() if isinstance(m, Qwen3ForCausalLM)), None)
    if lm is None:
        raise TypeError("apply_tensor_parallel: no Qwen3ForCausalLM inside the model")
    cfg = lm.config
    hq, hkv, f = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.intermediate_size
    assert hq % world == 0 and hkv % world == 0 and f % world == 0, \
        f"tp={world} must divide heads ({hq}/{hkv}) and intermediate size ({f})"
    if world == 1:
        return model
    lm.invalidate_fusion()
    for layer in lm.model.layers:
        a, mlp = layer.self_attn, layer.mlp
        for m in (a.q_proj, a.k_proj, a.v_proj):
            _shard_linear(m, 0, rank, world)
        _shard_linear(a.o_proj, 1, rank, world)
        a.hq, a.hkv = hq // world, hkv // world
        a.tp_group, a.tp_rank = group, rank
        for m in (mlp.gate_proj, mlp.up_proj):
            _shard_linear(m, 0, rank, world)
        _shard_linear(mlp.down_proj, 1, rank, world)
        mlp.tp_group, mlp.tp_rank = group, rank
    local = copy.copy(cfg)
    local.num_attention_heads = hq // world
    local.num_key_value_heads = hkv // world
    local.intermediate_size = f // world
    local.tp_size = world
    lm.config = local
    lm.model.cfg = local
    for layer in lm.model.layers:
        layer.self_attn.cfg = local
    return model
