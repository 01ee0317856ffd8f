"""Activations (K5).  SwiGLU over the fused ``[gate | up]`` projection output."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference as ref
from ._native import native, use_native, fn_apply


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(dy.contiguous(), gu)


def swiglu_fused(gu: torch.Tensor) -> torch.Tensor:
    """gu [T, 2F] = [gate | up] → silu(gate)·up [T, F]."""
    if use_native(gu):
        return fn_apply(_SwiGLUFn, gu.contiguous())
    f = gu.shape[-1] // 2
    return ref.swiglu(gu[..., :f], gu[..., f:])


class _GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return native().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return native().gelu_bwd(dy.contiguous(), x)


def gelu(x: torch.Tensor) -> torch.Tensor:
    """Exact (erf) GELU as ``nn.GELU()`` (``ddp_gpt_wikitext2.py:103``)."""
    if use_native(x) and x.is_contiguous():
        return fn_apply(_GeluFn, x)
    return F.gelu(x)
