"""Pipeline-parallel inference.

Reference: Ray Serve LLM with vLLM ``pipeline_parallel_size: 2`` over the ``ray`` executor and
``enforce_eager`` (``Deployment/Ray/serve_deploy_examples/qwen3_app_pipeline_parallel.yaml:21-31``;
README stance "TP within a node, PP across nodes", ``Deployment/Ray/README.md:358-362``).

Here: one process per GPU under ``torchrun``, the decoder layers split into contiguous stages
(balanced, earlier stages take the remainder); each stage keeps only its own layers and a KV
cache for them.  A forward step runs the stages in order — stage *s* receives the ``[tokens,
hidden]`` activations from stage *s−1* (``recv``), runs its layers and ``send``s them on — and
the last stage broadcasts its output to the whole PP group, so every rank applies the final
norm and LM head itself and the SPMD serving engine (``infer/engine.py``, same lockstep scheme
as tensor parallelism) samples identical tokens everywhere without a token exchange.
Composes with tensor parallelism: ``world = tp × pp``, stage = ``rank // tp``; the P2P links
join ranks with the same TP rank (:func:`make_tp_pp_groups`).

On one MI355X node the weights of every supported model fit a single GPU (288 GB), so PP is
the memory-scaling / multi-node option, not a throughput one: stages execute one after another
per step (no micro-batch interleave), like the reference's ``enforce_eager`` vLLM PP.
Inference only (training stays DDP / ZeRO, as in the reference).
"""
from __future__ import annotations

import copy

import torch
import torch.distributed as dist
import torch.nn as nn


def stage_bounds(n_layers: int, n_stages: int, stage: int) -> tuple[int, int]:
    """Layers ``[l0, l1)`` of ``stage``: contiguous, sizes differ by at most one."""
    base, extra = divmod(n_layers, n_stages)
    l0 = stage * base + min(stage, extra)
    return l0, l0 + base + (1 if stage < extra else 0)


class PipelineStageLink:
    """P2P hand-off of the residual stream between adjacent stages of one PP group."""

    def __init__(self, group, n_layers: int, global_l0: int):
        self.group = group
        self.stage = dist.get_rank(group)
        self.n_stages = dist.get_world_size(group)
        self.n_layers, self.l0 = n_layers, global_l0
        g = lambda r: dist.get_global_rank(group, r)   # noqa: E731
        self.prev = g(self.stage - 1) if self.stage > 0 else None
        self.next = g(self.stage + 1) if self.stage + 1 < self.n_stages else None
        self.last = g(self.n_stages - 1)

    def enter(self, x: torch.Tensor) -> torch.Tensor:
        if self.prev is None:
            return x
        buf = torch.empty_like(x)
        dist.recv(buf, src=self.prev, group=self.group)
        return buf

    def exit(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        if self.next is not None:
            dist.send(x, dst=self.next, group=self.group)
        if self.n_stages > 1:
            dist.broadcast(x, src=self.last, group=self.group)
        return x


def apply_pipeline_parallel(model: nn.Module, group=None) -> nn.Module:
    """Keep this rank's stage of a ``Qwen3ForCausalLM`` (in place) and link it to its
    neighbours in ``group`` (default: the world).  Embedding and LM head stay on every stage
    (the engine samples on every rank); the other stages' layers are freed."""
    if group is None:
        group = dist.group.WORLD
    n = dist.get_world_size(group)
    from ..models.qwen3 import Qwen3ForCausalLM
    lm = next((m for m in model.modules() if isinstance(m, Qwen3ForCausalLM)), None)
    if lm is None:
        raise TypeError("apply_pipeline_parallel: no Qwen3ForCausalLM inside the model")
    cfg = lm.config
    L = cfg.num_hidden_layers
    if n > L:
        raise ValueError(f"pp={n} stages for {L} layers")
    if n == 1:
        return model
    l0, l1 = stage_bounds(L, n, dist.get_rank(group))
    lm.invalidate_fusion()
    keep = list(lm.model.layers)[l0:l1]
    lm.model.layers = nn.ModuleList(keep)
    for i, layer in enumerate(keep):
        layer.self_attn.layer_idx = i       # KV cache rows of the local layers only
    local = copy.copy(cfg)
    local.num_hidden_layers = l1 - l0
    local.pp_size = n
    lm.config = local
    lm.model.cfg = local
    lm.model.pp = PipelineStageLink(group, L, l0)
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return model


def make_tp_pp_groups(tp: int, pp: int):
    """World = ``tp × pp`` ranks, stage = ``rank // tp``.  Returns ``(tp_group, pp_group)`` of
    this rank (``None`` for a degree of 1).  Every rank creates every group, in the same order."""
    world, rank = dist.get_world_size(), dist.get_rank()
    if tp * pp != world:
        raise ValueError(f"tensor_parallel_size {tp} x pipeline_parallel_size {pp} != world size {world}")
    if tp == world:
        return dist.group.WORLD, None
    if pp == world:
        return None, dist.group.WORLD
    tp_group = pp_group = None
    for s in range(pp):
        g = dist.new_group([s * tp + t for t in range(tp)])
        if rank // tp == s:
            tp_group = g
    for t in range(tp):
        g = dist.new_group([s * tp + t for s in range(pp)])
        if rank % tp == t:
            pp_group = g
    return tp_group, pp_group
