"""Embedding gather / gradient scatter-add on the HIP kernels of
``csrc/kernels/embedding.hip``.

:class:`Embedding` is a drop-in ``nn.Embedding`` (same ``weight`` parameter and state-dict key, so
checkpoints of the reference's models load unchanged) whose GPU forward is the row-gather kernel
and whose backward is the fp32 scatter-add kernel (cast to the table's dtype once).  CPU tensors,
``max_norm`` / ``sparse`` / ``scale_grad_by_freq`` and rows whose byte size is not a multiple of 16
use ``torch.nn.functional.embedding`` (the reference behaviour).  Reference usage:
``llm-demo/minigpt/model.py`` (token + position tables), ``GPTLike_wikitext2*.py`` (``tok_emb``,
learned ``pos_emb``), ``HF_Basics/trainer_demo.py`` (BERT word/position/type tables).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._native import native, use_native


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.V, ctx.pad, ctx.wdtype = weight.shape[0], padding_idx, weight.dtype
        return native().embedding_fwd(weight, ids)

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None
        d = dout if dout.dtype in (torch.bfloat16, torch.float32) else dout.float()
        gw = native().embedding_bwd(d, ids, ctx.V, -1 if ctx.pad is None else ctx.pad)
        return None, gw.to(ctx.wdtype), None


def _native_ok(ids: torch.Tensor, weight: torch.Tensor) -> bool:
    return (use_native(weight) and ids.dtype == torch.long and weight.dim() == 2
            and weight.shape[1] % 8 == 0 and (weight.shape[1] * weight.element_size()) % 16 == 0
            and weight.is_contiguous())


def embedding(ids: torch.Tensor, weight: torch.Tensor, padding_idx: int | None = None) -> torch.Tensor:
    if _native_ok(ids, weight):
        if not torch.is_grad_enabled() or not weight.requires_grad:
            return native().embedding_fwd(weight, ids)
        from .linear import deterministic
        if not deterministic():   # the scatter-add's fp32 atomics sum in arrival order
            return _EmbeddingFn.apply(ids, weight, padding_idx)
    return F.embedding(ids, weight, padding_idx)


class Embedding(nn.Embedding):
    """``nn.Embedding`` on the HIP gather / scatter-add kernels (see module docstring)."""

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if self.max_norm is not None or self.sparse or self.scale_grad_by_freq:
            return super().forward(ids)
        return embedding(ids, self.weight, self.padding_idx)
