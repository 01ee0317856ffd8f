"""Causal self-attention (K1): flash-style fused forward/backward on gfx950 MFMA.

API is token-major and head-interleaved: ``q [T, Hq*D]``, ``k/v [T, Hkv*D]`` where
``T = B*S``; k/v may be strided views into the fused qkv projection output (row stride
``(Hq+2Hkv)*D``) so no copy is made.  GQA is handled by head broadcast inside the kernel
(never materialising repeated K/V).  ``kv_lens`` ([B] int32) masks right padding.
The kernel also returns the per-row log-sum-exp so the backward recomputes P instead of
storing the S×S matrix; the API leaves room for a later ring/context-parallel merge
(SURVEY.md §5.7).
"""
from __future__ import annotations

import math

import torch

from . import reference as ref
from ._native import native, use_native


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, B, S, hq, hkv, d, causal, scale, kv_lens):
        o, lse = native().attn_fwd(q, k, v, kv_lens, B, S, hq, hkv, d, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse, kv_lens)
        ctx.meta = (B, S, hq, hkv, d, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kv_lens = ctx.saved_tensors
        B, S, hq, hkv, d, causal, scale = ctx.meta
        dq, dk, dv = native().attn_bwd(do.contiguous(), q, k, v, o, lse, kv_lens, B, S, hq, hkv, d, causal, scale)
        return dq, dk, dv, None, None, None, None, None, None, None, None


def flash_attention(q, k, v, batch: int, seqlen: int, hq: int, hkv: int, d: int,
                    causal: bool = True, scale: float | None = None,
                    kv_lens: torch.Tensor | None = None) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    if use_native(q) and d in (64, 128) and q.dtype == torch.bfloat16:
        return _FlashAttnFn.apply(q, k, v, batch, seqlen, hq, hkv, d, causal, scale, kv_lens)
    qb = q.reshape(batch, seqlen, hq, d)
    kb = k.reshape(batch, seqlen, hkv, d)
    vb = v.reshape(batch, seqlen, hkv, d)
    mask = None
    if kv_lens is not None:
        mask = torch.arange(seqlen, device=q.device)[None, :] < kv_lens[:, None]
    o = ref.attention(qb, kb, vb, causal=causal, key_padding_mask=mask, scale=scale)
    return o.reshape(batch * seqlen, hq * d)


def sdpa_bshd(q, k, v, causal=True, scale=None, dropout_p=0.0, window=None, key_padding_mask=None):
    """[B,S,H,D] convenience wrapper used by the small teaching models (GPTLike, MLA,
    notebook attention variants).  Routes to the fused kernel when shapes allow it."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    if (use_native(q) and q.dtype == torch.bfloat16 and dropout_p == 0.0 and window is None
            and key_padding_mask is None and k.shape[1] == S and D in (64, 128) and Hq % Hkv == 0
            and (S % 64 == 0 or not torch.is_grad_enabled())):
        o = flash_attention(q.reshape(B * S, Hq * D), k.reshape(B * S, Hkv * D).contiguous(),
                            v.reshape(B * S, Hkv * D).contiguous(), B, S, Hq, Hkv, D, causal, scale)
        return o.view(B, S, Hq, D)
    return ref.attention(q, k, v, causal=causal, scale=scale, dropout_p=dropout_p, window=window,
                         key_padding_mask=key_padding_mask)
