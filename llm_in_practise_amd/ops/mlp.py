"""SwiGLU MLP block with the activation fused into the GEMM epilogues.

    y = down( silu(x·W_gateᵀ) · (x·W_upᵀ) ) + residual

Unfused, the block is four kernels per direction: the gate|up GEMM writes gu [T, 2F], a SwiGLU
pass reads it back and writes h [T, F], the down GEMM reads h; in backward the down dX GEMM writes
dh, a SwiGLU-backward pass reads dh and gu and writes dgu.  Here (csrc/kernels/gemm4w.hip):

* forward: ONE gate|up launch writes gu (kept for backward) AND h — its B operand gathers gate and
  up rows so every lane holds g and u of the same (token, column) — then the down GEMM (+ residual);
* backward: ONE down-dX launch computes dh tile by tile and applies the SwiGLU backward in its
  epilogue from gu, writing dgu directly; then the gate|up dX GEMM.

Per Qwen3-8B layer at T = 2048 that removes two memory-bound passes (≈ 25 + 38 µs) and 150 MB of
HBM traffic, and h is not saved for backward (the frozen down base needs no weight gradient).

Used when nothing else sits between the GEMMs: no LoRA / multi-LoRA adapter on gate, up or down,
frozen bases (NF4 — read by the kernels as 4-bit codes, expanded per quant block inside the GEMM — or
bf16), training-sized token counts.  Otherwise the block runs as separate projections.
Reference: ``Fine-Tuning/qwen3-8b-qlora-dist.py:96-125`` (Qwen3 MLP under QLoRA, adapters on q/v).
"""
from __future__ import annotations

import torch

from ..quant.nf4 import NF4Weight
from ._native import native, fn_apply
from .checkpoint import _sac_recording, sac_put, sac_take, saves_discarded, tail_skippable
from .gemm import _MIN_M, _count, _nf4_expand, _nf4_w4


def _operand(base, reused: bool):
    """(weight, scale) as the gemm4w entry points take it: an NF4 base as its g4w-packed codes + the
    transposed block absmax (the kernel expands them) or as one bf16 expansion (ops/linear.py
    ``_nf4_w4`` decides), a bf16 base as itself with no scale."""
    if isinstance(base, NF4Weight):
        return base.g4w_pack() if _nf4_w4(reused) else (_nf4_expand(base), None)
    return base.contiguous(), None


def _form(scale) -> str:
    return "gemm4w" if scale is None else "gemm4w-nf4"


def fusable(x: torch.Tensor, gu_base, down_base, F: int, K: int) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and F % 64 == 0 and K % 64 == 0):
        return False
    if x.numel() // x.shape[-1] < _MIN_M:
        return False
    for b, shape in ((gu_base, (2 * F, K)), (down_base, (K, F))):
        if isinstance(b, NF4Weight):
            if tuple(b.shape) != shape or not b.kernel_ok():
                return False
        elif not (isinstance(b, torch.Tensor) and b.dtype == torch.bfloat16 and tuple(b.shape) == shape
                  and not b.requires_grad):
            return False
    return True


class _SwiGLUMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, bases):
        gu_base, down_base = bases
        K = x.shape[1]
        need = ctx.needs_input_grad[0]
        w_gu, s_gu = _operand(gu_base, need)
        w_d, s_d = _operand(down_base, need)
        replay = sac_take()       # selective checkpointing (ops/linear.py): the recorded (gu, y)
        if replay is not None:
            gu, y = replay
        else:
            F = gu_base.shape[0] // 2
            _count(_form(s_gu))
            # checkpointed layer: the recompute needs only gu (saved) — y, the layer output, feeds no saved tensor
            # (early stop) and with it h; the first forward needs h and y but drops what it saves, so not gu
            skip = tail_skippable(1 if need else 0)
            keep_gu = (need and not saves_discarded()) or _sac_recording()   # (selective: the stash replays gu)
            gu, h = native().gemm4w_swiglu(x, w_gu, s_gu, F, keep_gu, not skip)
            if skip:
                y = torch.empty_like(x)
            else:
                _count(_form(s_d))
                y = native().gemm4w(h, w_d, residual, 0, False, 0, 0, s_d, K)
            if need and gu is None:
                gu = x.new_empty(0)       # the placeholder a discarded save needs (same pack count as the recompute)
            sac_put((gu, y))
        ctx.save_for_backward(gu if need else None)
        ctx.w = (w_gu, s_gu, w_d, s_d, K) if need else None
        ctx.has_residual = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        dx = None
        if ctx.w is not None:
            w_gu, s_gu, w_d, s_d, K = ctx.w
            _count(_form(s_d))
            _count(_form(s_gu))
            dgu = native().gemm4w_dswiglu(dy.contiguous(), w_d, gu, s_d)
            dx = native().gemm4w(dgu, w_gu, None, 0, True, 0, 0, s_gu, K)
        ctx.w = None
        return dx, (dy if ctx.has_residual else None), None


def swiglu_mlp(x: torch.Tensor, gu_base, down_base, residual: torch.Tensor | None = None) -> torch.Tensor:
    """x [..., K] → down(silu(gate)·up) (+ residual) [..., K]; caller checked :func:`fusable`."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1]).contiguous()
    r2 = residual.reshape(-1, residual.shape[-1]).contiguous() if residual is not None else None
    y = fn_apply(_SwiGLUMLPFn, x2, r2, (gu_base, down_base))
    return y.view(*shape[:-1], y.shape[-1])
