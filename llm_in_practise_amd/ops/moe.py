"""MoE routing and token dispatch (reference: ``DeepSeekLike_wikitext2.py:276-309``
dense masked loop, ``DeepSeekLike_spare_MoE_wikitext2.py`` nonzero-gather + ``index_add_``).

On HIP tensors these run the ``moe.hip`` kernels (fused top-k/softmax routing, deterministic
stable permutation into contiguous per-expert segments, gather and gate-weighted combine with
fp32 accumulation — no atomics, no host sync until the per-expert GEMM loop reads the segment
offsets).  CPU tensors run the equivalent torch code below; both are autograd-complete.

    w, idx = moe_route(logits, k, mode)            # mode "topk_softmax" | "softmax_topk"
    d = moe_dispatch(idx, num_experts)             # pos_of [T·k], perm [T·k], offsets [E+1]
    xs = moe_gather(x, d)                          # [T·k, H] rows sorted by expert
    ys = expert_i(xs[off[i]:off[i+1]]) …           # per-expert GEMMs on contiguous slices
    out = moe_combine(ys, d, w, base)              # base + Σ_j w[t,j]·ys[pos_of[t,j]]
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn.functional as F

from ._native import native, use_native, fn_apply

_MODES = {"topk_softmax": 0, "softmax_topk": 1}


# ------------------------------------------------------------------ routing
class _RouteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, k, mode):
        idx, w, probs = native().moe_route(logits.contiguous(), k, mode, mode == 1)
        ctx.save_for_backward(w, idx, probs if mode == 1 else None)
        ctx.mode, ctx.E, ctx.dt = mode, logits.shape[1], logits.dtype
        ctx.mark_non_differentiable(idx)
        return w, idx

    @staticmethod
    def backward(ctx, dw, _didx):
        w, idx, probs = ctx.saved_tensors
        dl = native().moe_route_bwd(dw.float().contiguous(), w, idx, probs, ctx.E, ctx.mode, ctx.dt)
        return dl, None, None


def moe_route(logits: torch.Tensor, k: int, mode: str = "topk_softmax"):
    """Router logits [T, E] → (gate weights fp32 [T, k], expert ids [T, k]).

    ``topk_softmax``: top-k of the raw logits, softmax over the k (DeepSeekLike).
    ``softmax_topk``: softmax over all experts, top-k probabilities, unnormalised (notebook)."""
    m = _MODES[mode]
    if use_native(logits) and logits.shape[1] <= 64 and k <= 8:
        w, idx = fn_apply(_RouteFn, logits, k, m)
        return w, idx.long()
    if m == 1:
        w, idx = F.softmax(logits.float(), -1).topk(k, -1)
        return w, idx
    top, idx = logits.float().topk(k, -1)
    return F.softmax(top, -1), idx


# ------------------------------------------------------------------ permutation
@dataclasses.dataclass
class Dispatch:
    pos_of: torch.Tensor      # [T·k] row of pair (t, j) in the expert-sorted order
    perm: torch.Tensor        # [T·k] pair index of each sorted row (token = pair // k)
    offsets: torch.Tensor     # [E+1] segment starts (device)
    k: int

    def counts(self) -> list[int]:
        off = self.offsets.tolist()
        return [off[i + 1] - off[i] for i in range(len(off) - 1)]


def moe_dispatch(idx: torch.Tensor, num_experts: int) -> Dispatch:
    T, k = idx.shape
    flat = idx.reshape(-1)
    if use_native(idx):
        pos_of, perm, off = native().moe_permute(flat.to(torch.int32).contiguous(), num_experts)
        return Dispatch(pos_of, perm, off, k)
    perm = torch.argsort(flat, stable=True)
    pos_of = torch.empty_like(perm)
    pos_of[perm] = torch.arange(perm.numel(), device=perm.device)
    cnt = torch.bincount(flat, minlength=num_experts)
    off = torch.cat([cnt.new_zeros(1), cnt.cumsum(0)])
    return Dispatch(pos_of.int(), perm.int(), off.int(), k)


# ------------------------------------------------------------------ gather / combine
def _native_rows_ok(x):
    return x.dim() == 2 and x.shape[1] % 8 == 0 and x.dtype in (torch.float32, torch.bfloat16)


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos_of, perm, k):
        ctx.save_for_backward(pos_of)
        ctx.k = k
        return native().moe_gather(x.contiguous(), perm, k, None)

    @staticmethod
    def backward(ctx, dxs):
        (pos_of,) = ctx.saved_tensors
        return native().moe_combine(dxs.contiguous(), pos_of, ctx.k, None, None), None, None, None


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ys, w, base, pos_of, perm, k):
        ys = ys.contiguous()
        wf = w.float().contiguous()
        ctx.save_for_backward(ys, wf, pos_of, perm)
        ctx.k, ctx.has_base, ctx.wdt = k, base is not None, w.dtype
        return native().moe_combine(ys, pos_of, k, wf, base.contiguous() if base is not None else None)

    @staticmethod
    def backward(ctx, dout):
        ys, wf, pos_of, perm = ctx.saved_tensors
        dout = dout.contiguous()
        dys = native().moe_gather(dout, perm, ctx.k, wf.reshape(-1))
        dw = native().moe_wgrad(dout, ys, pos_of, ctx.k).to(ctx.wdt) if ctx.needs_input_grad[1] else None
        return dys, dw, (dout if ctx.has_base else None), None, None, None


def moe_gather(x: torch.Tensor, d: Dispatch) -> torch.Tensor:
    """x [T, H] → xs [T·k, H] with row p = x[perm[p] // k] (expert-sorted)."""
    if use_native(x) and _native_rows_ok(x):
        return fn_apply(_GatherFn, x, d.pos_of, d.perm, d.k)
    return x.index_select(0, (d.perm // d.k).long())


def moe_combine(ys: torch.Tensor, d: Dispatch, w: torch.Tensor, base: torch.Tensor | None = None) -> torch.Tensor:
    """out[t] = base[t] + Σ_j w[t, j] · ys[pos_of[t·k + j]]  (gate-weighted un-permute + sum)."""
    if use_native(ys) and _native_rows_ok(ys) and (base is None or base.dtype == ys.dtype):
        return fn_apply(_CombineFn, ys, w, base, d.pos_of, d.perm, d.k)
    T = d.pos_of.numel() // d.k
    g = ys.index_select(0, d.pos_of.long()).view(T, d.k, -1)
    out = (g * w.to(ys.dtype).unsqueeze(-1)).sum(1)
    return out if base is None else out + base
