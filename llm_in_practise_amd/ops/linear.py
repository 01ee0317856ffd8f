"""Frozen-base linear with LoRA fused into the base GEMM (K8) and NF4 dequant-GEMM (K9).

One op covers every projection of the stack:

    y[:, c0:c1] (+)= x · deq(W)ᵀ  +  Σ_i s_i · (drop_i(x) · A_iᵀ) · B_iᵀ   (+ residual)

* ``base`` is a bf16 ``[N, K]`` tensor (LoRA / full fine-tune) or an :class:`NF4Weight`
  (QLoRA).  Several projections that share an input (q|k|v, gate|up) are row-concatenated
  into one base and one GEMM; each LoRA branch owns a column range ``[c0, c1)``.
* On gfx950 the LoRA low-rank product is not a separate GEMM: ``s·x·Aᵀ`` ([T, Σr]) and the
  block-placed ``B`` ([N, Σr]) enter the MFMA kernel as an extra K-slice of the same tile
  loop (``gemm_nf4`` / ``gemm_bf16`` in ``csrc/kernels/gemm_*.hip``), and the residual add
  is the epilogue.  Backward ``dX = dY·deq(W)`` is the transposed-operand variant of the
  same kernel (the NF4 tile is dequantised into LDS and read back transposed), with the
  LoRA ``(s·dY·B)·A`` term again an extra K-slice when the branch has no dropout.

Reference parity: PEFT ``LoraConfig(r, lora_alpha, lora_dropout, target_modules)``
(``Fine-Tuning/qwen3-8b-qlora.py:107-114``), scaling = alpha / r.
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn.functional as F

from ..quant.nf4 import NF4Weight, dequantize_nf4
from ._native import native, use_native

EXT_ALIGN = 32   # the kernels consume the LoRA K-slice in MFMA K-steps of 32


@dataclasses.dataclass
class LoraBranch:
    a: torch.Tensor          # [r, K]
    b: torch.Tensor          # [n, r]
    scaling: float
    dropout: float
    c0: int
    c1: int


def _pad_cols(t: torch.Tensor, mult: int = EXT_ALIGN) -> torch.Tensor:
    r = t.shape[-1]
    rp = (r + mult - 1) // mult * mult
    if rp == r:
        return t.contiguous()
    return F.pad(t, (0, rp - r)).contiguous()


def _base_gemm(x, base, ext_a=None, ext_b=None, residual=None):
    if isinstance(base, NF4Weight):
        if not base.kernel_ok():      # odd shapes: dequantise then library GEMM
            y = x @ dequantize_nf4(base, x.dtype).t()
            if ext_a is not None:
                y = y + ext_a @ ext_b.t()
            return y if residual is None else y + residual
        cf, _, at = base.kernel_pack()
        return native().gemm_nf4(x, cf, at, base.shape[0], ext_a, ext_b, residual)
    return native().gemm_bf16(x, base, ext_a, ext_b, residual)


def _base_gemm_t(dy, base, ext_a=None, ext_b=None):
    """dX = dY·W (+ ext_a · ext_bᵀ, ext_b given as [K, R])."""
    if isinstance(base, NF4Weight):
        if not base.kernel_ok():
            dx = dy @ dequantize_nf4(base, dy.dtype)
            return dx if ext_a is None else dx + ext_a @ ext_b.t()
        _, cb, at = base.kernel_pack()
        return native().gemm_nf4_t(dy, cb, at, base.shape[1], ext_a, ext_b)
    return native().gemm_bf16_t(dy, base, ext_a, ext_b)


class _FusedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, meta, *ab):
        base, branches, training = meta
        dense = not isinstance(base, NF4Weight)
        xa_list, xd_list, mask_list = [], [], []
        ext_a = ext_b = None
        if branches:
            N = base.shape[0]
            rtot = sum(br.a.shape[0] for br in branches)
            ext_b = x.new_zeros(N, (rtot + EXT_ALIGN - 1) // EXT_ALIGN * EXT_ALIGN)
            cols, r0 = [], 0
            for br, (a, b) in zip(branches, zip(ab[0::2], ab[1::2])):
                r = a.shape[0]
                if training and br.dropout > 0:
                    mask = torch.rand_like(x, dtype=torch.float32).ge_(br.dropout)
                    xd = x * mask.to(x.dtype) * (1.0 / (1.0 - br.dropout))
                else:
                    mask, xd = None, x
                xa = xd @ a.to(x.dtype).t()                       # [T, r]
                cols.append(xa * br.scaling)
                ext_b[br.c0:br.c1, r0:r0 + r] = b.to(x.dtype)
                xa_list.append(xa)
                xd_list.append(xd if mask is not None else None)
                mask_list.append(mask)
                r0 += r
            ext_a = _pad_cols(torch.cat(cols, 1))
        y = _base_gemm(x, base if not dense else weight, ext_a, ext_b, residual)
        if bias is not None:
            y = y + bias
        ctx.meta = meta
        ctx.has_residual = residual is not None
        ctx.save_for_backward(x, weight, *ab, *[t for t in xa_list],
                              *[t if t is not None else torch.empty(0) for t in xd_list],
                              *[t if t is not None else torch.empty(0) for t in mask_list])
        ctx.nb = len(branches)
        return y

    @staticmethod
    def backward(ctx, dy):
        base, branches, training = ctx.meta
        saved = ctx.saved_tensors
        x, weight = saved[0], saved[1]
        nb = ctx.nb
        ab = saved[2:2 + 2 * nb]
        xa_list = saved[2 + 2 * nb:2 + 3 * nb]
        xd_list = saved[2 + 3 * nb:2 + 4 * nb]
        mask_list = saved[2 + 4 * nb:2 + 5 * nb]
        dense = not isinstance(base, NF4Weight)
        dy = dy.contiguous()
        grads_ab = []
        g_list = []
        for i, br in enumerate(branches):
            a, b = ab[2 * i], ab[2 * i + 1]
            dyi = dy[:, br.c0:br.c1]
            g = (dyi @ b.to(dy.dtype)) * br.scaling            # [T, r]  = d(xa)
            db = (dyi.t() @ xa_list[i]) * br.scaling           # [n, r]
            xin = xd_list[i] if xd_list[i].numel() else x
            da = g.t() @ xin                                   # [r, K]
            grads_ab += [da.to(a.dtype), db.to(b.dtype)]
            g_list.append(g)
        dx = None
        if ctx.needs_input_grad[0]:
            fold = [i for i, br in enumerate(branches) if not mask_list[i].numel()]
            ext_a = ext_b = None
            if fold:
                ext_a = _pad_cols(torch.cat([g_list[i] for i in fold], 1))
                ext_b = torch.cat([ab[2 * i].to(dy.dtype) for i in fold], 0)            # [R, K]
                ext_b = F.pad(ext_b, (0, 0, 0, ext_a.shape[1] - ext_b.shape[0])).t().contiguous()  # [K, Rp]
            dx = _base_gemm_t(dy, base if not dense else weight, ext_a, ext_b)
            for i, br in enumerate(branches):
                if mask_list[i].numel():
                    scale = 1.0 / (1.0 - br.dropout)
                    dx.addcmul_(g_list[i] @ ab[2 * i].to(dy.dtype), mask_list[i].to(dy.dtype), value=scale)
        dres = dy if ctx.has_residual else None
        dw = None
        if dense and weight is not None and ctx.needs_input_grad[2]:
            dw = (dy.t() @ x).to(weight.dtype)
        dbias = dy.sum(0) if ctx.needs_input_grad[3] else None
        return (dx, dres, dw, dbias, None, *grads_ab)


def _reference(x, base, bias, branches, residual, training):
    w = dequantize_nf4(base, x.dtype) if isinstance(base, NF4Weight) else base
    y = x @ w.to(x.dtype).t()
    if branches:
        extra = torch.zeros_like(y)
        for br in branches:
            xd = F.dropout(x, br.dropout, training=training) if br.dropout > 0 else x
            upd = (xd @ br.a.to(x.dtype).t()) @ br.b.to(x.dtype).t() * br.scaling
            extra = extra.index_add(1, torch.arange(br.c0, br.c1, device=x.device), upd)
        y = y + extra
    if bias is not None:
        y = y + bias
    if residual is not None:
        y = y + residual
    return y


def fused_linear(x: torch.Tensor, base, bias: torch.Tensor | None = None,
                 branches: list[LoraBranch] | tuple = (), residual: torch.Tensor | None = None,
                 training: bool = True) -> torch.Tensor:
    """x [..., K] → [..., N].  See module docstring."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    res2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
    if use_native(x2) and x2.dtype == torch.bfloat16:
        weight = None if isinstance(base, NF4Weight) else base
        ab = []
        for br in branches:
            ab += [br.a, br.b]
        y = _FusedLinearFn.apply(x2.contiguous(), None if res2 is None else res2.contiguous(),
                                 weight, bias, (base, tuple(branches), training), *ab)
    else:
        y = _reference(x2, base, bias, branches, res2, training)
    return y.view(*shape[:-1], y.shape[-1])
