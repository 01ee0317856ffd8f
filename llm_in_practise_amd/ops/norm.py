"""RMSNorm / LayerNorm (K2, K4).  One-pass row-reduce HIP kernels on gfx950."""
from __future__ import annotations

import torch
import torch.nn as nn

from . import reference as ref
from ._native import native, use_native, fn_apply


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, rstd = native().rmsnorm_fwd(x2, weight, eps)
        ctx.save_for_backward(x2, rstd)
        ctx.weight = weight         # a parameter: no saved-tensor hook (non-reentrant checkpointing)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        (x2, rstd), weight = ctx.saved_tensors, ctx.weight
        need_dw = weight is not None and ctx.needs_input_grad[1]
        dx, dw = native().rmsnorm_bwd(dy.reshape(x2.shape).contiguous(), x2, weight, rstd, need_dw, None)
        return dx.view(ctx.shape), (dw.to(weight.dtype) if need_dw else None), None


class _RMSNormResidualFn(torch.autograd.Function):
    """(norm(x), x): x feeds both the pre-norm branch and the skip connection.  Returning the
    skip path from the same node lets backward fold the skip gradient into the norm backward
    kernel (one pass: dx = norm_bwd(dy_norm) + dy_skip) instead of autograd cloning one
    gradient and adding the other (two extra [T, hidden] passes per norm)."""

    @staticmethod
    def forward(ctx, x, weight, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, rstd = native().rmsnorm_fwd(x2, weight, eps)
        ctx.save_for_backward(x2, rstd)
        ctx.weight = weight
        ctx.shape = shape
        return y.view(shape), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        (x2, rstd), weight = ctx.saved_tensors, ctx.weight
        need_dw = weight is not None and ctx.needs_input_grad[1]
        if dy is None:
            return dskip, None, None
        dres = None if dskip is None else dskip.reshape(x2.shape).contiguous()
        dx, dw = native().rmsnorm_bwd(dy.reshape(x2.shape).contiguous(), x2, weight, rstd, need_dw, dres)
        return dx.view(ctx.shape), (dw.to(weight.dtype) if need_dw else None), None


def rms_norm(x: torch.Tensor, weight: torch.Tensor | None, eps: float = 1e-6) -> torch.Tensor:
    if use_native(x):
        return fn_apply(_RMSNormFn, x, weight, eps)
    return ref.rmsnorm(x, weight, eps)


def rms_norm_residual(x: torch.Tensor, weight: torch.Tensor | None, eps: float = 1e-6):
    """Pre-norm block entry: returns ``(rmsnorm(x), skip)`` where ``skip`` is ``x`` for the
    residual add; on the GPU the two gradients meet inside the norm backward kernel."""
    if use_native(x):
        return fn_apply(_RMSNormResidualFn, x, weight, eps)
    return ref.rmsnorm(x, weight, eps), x


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = native().layernorm_fwd(x2, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.shape = shape
        ctx.has_bias = bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        need_dw = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dx, dw, db = native().layernorm_bwd(dy.reshape(x2.shape).contiguous(), x2, weight, mean, rstd, need_dw)
        return (dx.view(ctx.shape), dw.to(weight.dtype) if need_dw else None,
                db.to(weight.dtype) if (need_dw and ctx.has_bias) else None, None)


def layer_norm(x, weight, bias, eps: float = 1e-5):
    if use_native(x):
        return fn_apply(_LayerNormFn, x, weight, bias, eps)
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)


class RMSNorm(nn.Module):
    """Qwen3 ``RMSNorm`` (input/post-attention/final norms and per-head q/k norms)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        return rms_norm(x, self.weight, self.eps)


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` with the gfx950 kernel underneath (GPTLike / MiniGPT blocks)."""

    def forward(self, x):
        return layer_norm(x, self.weight, self.bias, self.eps)
