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

from ._native import native, use_native, fn_apply


# Out-of-range token ids: F.embedding (the reference's op) raises; the gather kernel reads a clamped
# row (memory-safe) and sets a per-device error word that is checked lazily — the word copied at
# the previous call is examined at the next one (no host sync on the hot path), so a tokenizer /
# vocabulary mismatch fails within one step instead of training on wrong rows.
_OOB: dict = {}


def _oob_state(dev: torch.device):
    st = _OOB.get(dev)
    if st is None:
        st = _OOB[dev] = [torch.zeros(1, dtype=torch.int32, device=dev),
                          torch.zeros(1, dtype=torch.int32, pin_memory=True), None]
    return st


def check_ids() -> None:
    """Synchronously raise if any gather so far read an out-of-range id (and reset the word)."""
    for st in _OOB.values():
        bad = int(st[0].item())
        st[0].zero_()
        st[2] = None
        if bad:
            raise IndexError("embedding: token id out of range of the embedding table")


def _gather(weight, ids):
    dev = weight.device
    if torch.cuda.is_current_stream_capturing():     # graph capture: flag only, checked at the next eager call
        return native().embedding_fwd(weight, ids, _oob_state(dev)[0])
    st = _oob_state(dev)
    word, host, ev = st
    if ev is not None:                  # the copy queued behind the PREVIOUS gather: long complete
        ev.synchronize()
        st[2] = None
        if int(host[0]):
            word.zero_()
            raise IndexError("embedding: token id out of range of the embedding table (reported at the next call)")
    out = native().embedding_fwd(weight, ids, word)
    host.copy_(word, non_blocking=True)
    st[2] = torch.cuda.Event()
    st[2].record()
    return out


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ctx.save_for_backward(ids)
        ctx.V, ctx.pad, ctx.wdtype = weight.shape[0], padding_idx, weight.dtype
        return _gather(weight, ids)

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
            return _gather(weight, ids)
        from .linear import deterministic
        if not deterministic():   # the scatter-add's fp32 atomics sum in arrival order
            return fn_apply(_EmbeddingFn, ids, weight, padding_idx)
    return F.embedding(ids, weight, padding_idx)


class Embedding(nn.Embedding):
    """``nn.Embedding`` on the HIP gather / scatter-add kernels (see module docstring)."""

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if self.max_norm is not None or self.sparse or self.scale_grad_by_freq:
            return super().forward(ids)
        return embedding(ids, self.weight, self.padding_idx)
