"""Fused attention (K1): flash-style forward/backward on gfx950 MFMA.

API is token-major and head-interleaved: ``q [T, Hq*D]``, ``k/v [T, Hkv*D]`` where
``T = B*S``; k/v may be strided views into the fused qkv projection output (row stride
``(Hq+2Hkv)*D``) so no copy is made.  GQA is handled by head broadcast inside the kernel
(never materialising repeated K/V).  ``kv_lens`` ([B] int32) masks right padding (also BERT's
key-padding mask when it is a right-padding prefix).  Any sequence length, head_dim ∈
{32, 64, 96, 128}, optional attention-probability dropout (counter-RNG, regenerated in the
backward — ``nn.MultiheadAttention(dropout=p)`` of the teaching models,
``LLM_Distributed_Trainning/PyTorch/ddp_basics/ddp_gpt_wikitext2.py:89-96``).

:func:`flash_attention_prefix` is the inference form for chunked prefill and prefix-cache
suffix prefill: ``Sq`` new queries per row at absolute positions ``q_offs[b] + i`` over a KV cache
of ``Skv`` rows (``Fine-Tuning/README.md`` vLLM APC / chunked prefill parity).

The kernel returns the per-row log-sum-exp so the backward recomputes P instead of storing the
S×S matrix.
"""
from __future__ import annotations

import math

import torch

from . import reference as ref
from ._native import native, use_native, fn_apply

HEAD_DIMS = (32, 64, 96, 128)
_SEED = [0x243F6A8885A308D3]


def _next_seed() -> int:
    _SEED[0] = (_SEED[0] * 6364136223846793005 + 1442695040888963407) & 0x7FFFFFFFFFFFFFFF
    return _SEED[0]


def seed_attention_dropout(seed: int):
    _SEED[0] = (int(seed) * 0x2545F4914F6CDD1D) & 0x7FFFFFFFFFFFFFFF


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, B, S, hq, hkv, d, causal, scale, kv_lens, p_drop, seed):
        o, lse = native().attn_fwd_ext(q, k, v, kv_lens, None, B, S, S, S, hq, hkv, d, causal, scale, p_drop, seed)
        ctx.save_for_backward(q, k, v, o, lse, kv_lens)
        ctx.meta = (B, S, hq, hkv, d, causal, scale, p_drop, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kv_lens = ctx.saved_tensors
        B, S, hq, hkv, d, causal, scale, p_drop, seed = ctx.meta
        dq, dk, dv = native().attn_bwd(do.contiguous(), q, k, v, o, lse, kv_lens, B, S, hq, hkv, d, causal, scale,
                                       p_drop, seed)
        return dq, dk, dv, None, None, None, None, None, None, None, None, None, None


def _aligned(t: torch.Tensor, d: int = 0) -> bool:
    """Operand layout the kernels take: unit inner stride, 16-B aligned rows; at head_dim 128 (the LDS-DMA
    kernels) row strides in whole 256-B units."""
    return (t.stride(-1) == 1 and t.stride(0) % (128 if d == 128 else 8) == 0 and t.data_ptr() % 16 == 0)


def native_ok(q, d: int) -> bool:
    return use_native(q) and d in HEAD_DIMS and q.dtype == torch.bfloat16


def flash_attention(q, k, v, batch: int, seqlen: int, hq: int, hkv: int, d: int,
                    causal: bool = True, scale: float | None = None,
                    kv_lens: torch.Tensor | None = None, dropout_p: float = 0.0,
                    seed: int | None = None) -> torch.Tensor:
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    if native_ok(q, d):
        if not (_aligned(q, d) and _aligned(k, d) and _aligned(v, d)):
            q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        seed = _next_seed() if (dropout_p > 0 and seed is None) else (seed or 0)
        return fn_apply(_FlashAttnFn, q, k, v, batch, seqlen, hq, hkv, d, causal, scale, kv_lens, float(dropout_p), seed)
    qb = q.reshape(batch, seqlen, hq, d)
    kb = k.reshape(batch, seqlen, hkv, d)
    vb = v.reshape(batch, seqlen, hkv, d)
    mask = None
    if kv_lens is not None:
        mask = torch.arange(seqlen, device=q.device)[None, :] < kv_lens[:, None]
    o = ref.attention(qb, kb, vb, causal=causal, key_padding_mask=mask, scale=scale, dropout_p=dropout_p)
    return o.reshape(batch * seqlen, hq * d)


@torch.no_grad()
def flash_attention_prefix(q, k_cache, v_cache, batch: int, sq: int, skv: int, hq: int, hkv: int, d: int,
                           q_offs: torch.Tensor | int = 0, kv_lens: torch.Tensor | None = None,
                           scale: float | None = None, kv_rows: int | None = None) -> torch.Tensor:
    """Causal attention of ``sq`` new queries per row (``q [B*sq, Hq*D]``) over a KV cache
    ``k_cache/v_cache [B, kv_rows, Hkv*D]`` (first ``skv`` rows visible).  Query i of row b sits at
    position ``q_offs[b] + i`` and sees keys ``≤ q_offs[b] + i`` and ``< kv_lens[b]``."""
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    kv_rows = kv_rows if kv_rows is not None else k_cache.shape[1]
    if isinstance(q_offs, int):
        q_offs = torch.full((batch,), q_offs, dtype=torch.int32, device=q.device)
    if native_ok(q, d):
        kc = k_cache.reshape(batch * kv_rows, -1)
        vc = v_cache.reshape(batch * kv_rows, -1)
        if not _aligned(q, d):
            q = q.contiguous()
        if not (_aligned(kc, d) and _aligned(vc, d)):
            kc, vc = kc.contiguous(), vc.contiguous()
        o, _ = native().attn_fwd_ext(q, kc, vc, kv_lens, q_offs, batch, sq, skv, kv_rows, hq, hkv, d, True, scale,
                                     0.0, 0)
        return o
    kq = k_cache[:, :skv].reshape(batch, skv, hkv, d).float()
    vq = v_cache[:, :skv].reshape(batch, skv, hkv, d).float()
    qf = q.reshape(batch, sq, hq, d).float()
    pos_q = q_offs.to(q.device).long()[:, None] + torch.arange(sq, device=q.device)[None]      # [B, sq]
    keys = torch.arange(skv, device=q.device)
    allowed = keys[None, None, :] <= pos_q[:, :, None]                                           # [B, sq, skv]
    if kv_lens is not None:
        allowed &= keys[None, None, :] < kv_lens.to(q.device).long()[:, None, None]
    rep = hq // hkv
    kq = kq.repeat_interleave(rep, 2)
    vq = vq.repeat_interleave(rep, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kq) * scale
    s = s.masked_fill(~allowed[:, None], float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    o = torch.einsum("bhqk,bkhd->bqhd", p, vq)
    return o.reshape(batch * sq, hq * d).to(q.dtype)


def _right_pad_lengths(mask: torch.Tensor) -> torch.Tensor | None:
    """[B, S] bool key mask (True = attend) → per-row lengths when it is a right-padding prefix."""
    lens = mask.sum(1)
    if torch.equal(mask, torch.arange(mask.shape[1], device=mask.device)[None] < lens[:, None]):
        return lens.to(torch.int32)
    return None


def sdpa_bshd(q, k, v, causal=True, scale=None, dropout_p=0.0, window=None, key_padding_mask=None):
    """[B,S,H,D] attention for the teaching / pretraining families (GPTLike, BERT, MLA latent heads,
    the notebook variants).  Routes to the fused kernel whenever the shapes allow it (any S, any
    head_dim in {32, 64, 96, 128}, dropout, right-padding key masks); bf16 and fp16 activations
    run it in bf16 (fp16 is cast in and out).  fp32 models keep the exact fp32 reference.
    ``key_padding_mask`` is True where a key is VALID."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    if (use_native(q) and q.dtype in (torch.bfloat16, torch.float16) and window is None and k.shape[1] == S
            and D in HEAD_DIMS and Hq % Hkv == 0):
        kv_lens = None
        if key_padding_mask is not None:
            kv_lens = _right_pad_lengths(key_padding_mask.bool())
        if key_padding_mask is None or kv_lens is not None:
            dt = q.dtype
            cast = (lambda t: t.to(torch.bfloat16)) if dt != torch.bfloat16 else (lambda t: t)  # noqa: E731
            o = flash_attention(cast(q).reshape(B * S, Hq * D), cast(k).reshape(B * S, Hkv * D),
                                cast(v).reshape(B * S, Hkv * D), B, S, Hq, Hkv, D, causal, scale,
                                kv_lens=kv_lens, dropout_p=dropout_p)
            return o.view(B, S, Hq, D).to(dt)
    return ref.attention(q, k, v, causal=causal, scale=scale, dropout_p=dropout_p, window=window,
                         key_padding_mask=key_padding_mask)
