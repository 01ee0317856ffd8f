"""Cross-entropy (K7) and the fused, chunked LM-head + cross-entropy.

``fused_linear_cross_entropy`` never materialises the full ``[T, V]`` fp32 logits (1.2 GB
per 2 K tokens at V=151,936): per token chunk it runs the head GEMM (the hand-written MFMA
kernel of csrc/kernels/gemm4w.hip), then ONE HIP kernel computes the row log-sum-exp, the loss and overwrites
the bf16 logits with dlogits in place; ``dX`` for the chunk is one more GEMM.  The
gradient is produced during the forward (the loss is terminal), so the backward only
scales it.  Matches HF's causal-LM loss: labels shifted by one, ``ignore_index=-100``,
mean over valid tokens.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference as ref
from ._native import native, use_native, fn_apply
from .gemm import _count, _g4w_ok


def cross_entropy(logits, labels, ignore_index: int = -100):
    return ref.cross_entropy(logits, labels, ignore_index)


class _FusedLinearCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, labels, ignore_index, chunk, need_wgrad, groups):
        """``groups`` > 1: the rows are ``groups`` equal gradient-accumulation micro-batches and the
        loss is the mean of their per-micro-batch mean losses (row scale 1/(G·n_valid_g)), so
        the LM head runs as ONE larger GEMM instead of G smaller ones."""
        T = h.shape[0]
        valid = (labels != ignore_index).view(groups, -1).sum(1).clamp_min(1).float()
        inv = 1.0 / (valid * groups)                                # [G] per-row-group loss scale
        rows_g = T // groups
        if chunk % rows_g and groups > 1:
            chunk = rows_g * max(1, chunk // rows_g)               # chunks hold whole micro-batches
        dh = torch.empty_like(h)
        dw = torch.zeros(weight.shape, dtype=torch.float32, device=h.device) if need_wgrad else None
        loss = torch.zeros((), dtype=torch.float32, device=h.device)
        for s in range(0, T, chunk):
            hc = h[s:s + chunk]
            g4w = _g4w_ok(hc, weight, False)
            _count("gemm4w" if g4w else "library")
            logits = native().gemm4w(hc, weight, None, 0, False) if g4w else hc @ weight.t()
            g0, g1 = s // rows_g, (s + hc.shape[0]) // rows_g
            row_loss = native().ce_fwd_bwd(logits, labels[s:s + chunk], ignore_index, inv[g0:g1])
            loss += (row_loss.view(g1 - g0, -1).sum(1) * inv[g0:g1]).sum()
            dx_g4w = g4w and _g4w_ok(logits, weight, True)
            _count("gemm4w" if dx_g4w else "library")
            if dx_g4w:
                dhc = native().gemm4w(logits, weight, None, 0, True)
                if hc.shape[0] == T:
                    dh = dhc
                else:
                    dh[s:s + chunk] = dhc
            else:
                torch.matmul(logits, weight, out=dh[s:s + chunk])
            if need_wgrad:
                dw.add_(logits.t().float() @ hc.float())
        ctx.save_for_backward(dh, dw)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        dh, dw = ctx.saved_tensors
        return ((dh * gloss.to(dh.dtype)), (None if dw is None else (dw * gloss).to(torch.bfloat16)),
                None, None, None, None, None)


def fused_linear_cross_entropy(h: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                               ignore_index: int = -100, chunk: int = 4096, groups: int = 1) -> torch.Tensor:
    """mean CE of ``h @ weightᵀ`` against ``labels`` (already shifted), h [T, d].  With
    ``groups`` = G the rows are G equal micro-batches and the result is the mean over micro-batches
    of each one's mean loss (gradient-accumulation semantics)."""
    if use_native(h):
        need_w = weight.requires_grad
        return fn_apply(_FusedLinearCEFn, h.contiguous(), weight, labels.contiguous(), ignore_index, chunk, need_w,
                                      groups)
    _count("library")
    logits = h.float() @ weight.float().t()
    if groups == 1:
        return F.cross_entropy(logits, labels, ignore_index=ignore_index)
    lg, lb = logits.view(groups, -1, logits.shape[-1]), labels.view(groups, -1)
    return sum(F.cross_entropy(lg[g], lb[g], ignore_index=ignore_index) for g in range(groups)) / groups


def shift_labels(labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """HF causal-LM convention: position t predicts token t+1; last position ignored."""
    out = torch.full_like(labels, ignore_index)
    out[..., :-1] = labels[..., 1:]
    return out
