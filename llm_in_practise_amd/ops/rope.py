"""Rotary position embedding (K3) and the fused Qwen3 q/k-RMSNorm + RoPE op.

Layouts: activations are token-major ``[T, H*D]`` (T = batch*seq); cos/sin are gathered
per token ``[T, D/2]`` fp32 so arbitrary ``position_ids`` (training, KV-cache decode,
YaRN-scaled tables) go through one kernel.
"""
from __future__ import annotations

import torch

from . import reference as ref
from ._native import native, use_native, fn_apply


def _ref_rope_tok(x, cos, sin, interleaved):
    # x [T, H, D]; cos/sin [T, D/2]
    return ref.apply_rope(x, cos, sin, interleaved)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, interleaved):
        ctx.cs = (cos, sin)          # per-step constants: no saved-tensor hooks
        ctx.interleaved = interleaved
        return native().rope(x.contiguous(), cos, sin, interleaved, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.cs
        return native().rope(dy.contiguous(), cos, sin, ctx.interleaved, True), None, None, None


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, interleaved: bool = False):
    """x [T, H, D] (or [B, S, H, D] with cos/sin [B*S, D/2])."""
    shape = x.shape
    x3 = x.reshape(-1, shape[-2], shape[-1])
    if use_native(x):
        return fn_apply(_RopeFn, x3, cos, sin, interleaved).view(shape)
    return _ref_rope_tok(x3, cos, sin, interleaved).view(shape)


class _QKNormRopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, qw, kw, cos, sin, hq, hkv, d, eps):
        q, k, rq, rk = native().qk_norm_rope_fwd(qkv, qw, kw, cos, sin, hq, hkv, d, eps)
        ctx.save_for_backward(qkv, rq, rk)
        ctx.consts = (qw, kw, cos, sin)   # parameters / per-step tables: no saved-tensor hooks
        ctx.dims = (hq, hkv, d)
        v = qkv[:, (hq + hkv) * d:]
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        qkv, rq, rk = ctx.saved_tensors
        qw, kw, cos, sin = ctx.consts
        hq, hkv, d = ctx.dims
        dqkv = native().qk_norm_rope_bwd(dq.contiguous(), dk.contiguous(),
                                         None if dv is None else dv.contiguous(), qkv, qw, kw, cos, sin, rq, rk, hq, hkv, d)
        return dqkv, None, None, None, None, None, None, None, None


def qk_norm_rope(qkv: torch.Tensor, q_weight, k_weight, cos, sin, hq: int, hkv: int, d: int,
                 eps: float = 1e-6):
    """Split fused ``qkv [T, (hq+2hkv)*d]``; RMS-normalise each q/k head (Qwen3 qk-norm) and
    rotate (rotate-half).  Returns q ``[T, hq*d]``, k ``[T, hkv*d]``, v (strided view)."""
    if use_native(qkv):
        return fn_apply(_QKNormRopeFn, qkv.contiguous(), q_weight, k_weight, cos, sin, hq, hkv, d, eps)
    T = qkv.shape[0]
    q = qkv[:, : hq * d].reshape(T, hq, d)
    k = qkv[:, hq * d:(hq + hkv) * d].reshape(T, hkv, d)
    v = qkv[:, (hq + hkv) * d:]
    if q_weight is not None:
        q = ref.rmsnorm(q, q_weight, eps)
        k = ref.rmsnorm(k, k_weight, eps)
    q = ref.apply_rope(q, cos, sin)
    k = ref.apply_rope(k, cos, sin)
    return q.reshape(T, hq * d), k.reshape(T, hkv * d), v
