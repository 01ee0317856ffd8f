"""Cross-entropy (K7) and the fused, chunked LM-head + cross-entropy.

``fused_linear_cross_entropy`` never materialises the full ``[T, V]`` fp32 logits (1.2 GB
per 2 K tokens at V=151,936): per token chunk it runs the head GEMM (hipBLASLt, plain
library GEMM), then ONE HIP kernel computes the row log-sum-exp, the loss and overwrites
the bf16 logits with dlogits in place; ``dX`` for the chunk is one more GEMM.  The
gradient is produced during the forward (the loss is terminal), so the backward only
scales it.  Matches HF's causal-LM loss: labels shifted by one, ``ignore_index=-100``,
mean over valid tokens.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import reference as ref
from ._native import native, use_native


def cross_entropy(logits, labels, ignore_index: int = -100):
    return ref.cross_entropy(logits, labels, ignore_index)


class _FusedLinearCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, labels, ignore_index, chunk, need_wgrad):
        T = h.shape[0]
        n_valid = (labels != ignore_index).sum().clamp_min(1)
        inv = 1.0 / n_valid.float()
        dh = torch.empty_like(h)
        dw = torch.zeros(weight.shape, dtype=torch.float32, device=h.device) if need_wgrad else None
        loss_sum = torch.zeros((), dtype=torch.float32, device=h.device)
        for s in range(0, T, chunk):
            hc = h[s:s + chunk]
            logits = hc @ weight.t()                               # [c, V] bf16 (hipBLASLt)
            row_loss = native().ce_fwd_bwd(logits, labels[s:s + chunk], ignore_index, inv)
            loss_sum += row_loss.sum()
            torch.matmul(logits, weight, out=dh[s:s + chunk])      # dlogits @ W
            if need_wgrad:
                dw.add_(logits.t().float() @ hc.float())
        ctx.save_for_backward(dh, dw)
        return loss_sum * inv

    @staticmethod
    def backward(ctx, gloss):
        dh, dw = ctx.saved_tensors
        return (dh * gloss.to(dh.dtype)), (None if dw is None else (dw * gloss).to(torch.bfloat16)), None, None, None, None


def fused_linear_cross_entropy(h: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor,
                               ignore_index: int = -100, chunk: int = 2048) -> torch.Tensor:
    """mean CE of ``h @ weightᵀ`` against ``labels`` (already shifted), h [T, d]."""
    if use_native(h):
        need_w = weight.requires_grad
        return _FusedLinearCEFn.apply(h.contiguous(), weight, labels.contiguous(), ignore_index, chunk, need_w)
    logits = h.float() @ weight.float().t()
    return F.cross_entropy(logits, labels, ignore_index=ignore_index)


def shift_labels(labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """HF causal-LM convention: position t predicts token t+1; last position ignored."""
    out = torch.full_like(labels, ignore_index)
    out[..., :-1] = labels[..., 1:]
    return out
