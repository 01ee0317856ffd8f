"""Transformer building blocks for the teaching models.

Parameter names mirror ``torch.nn`` (``in_proj_weight``, ``out_proj``, ``linear1``, ``norm1`` …)
so state dicts saved by the reference scripts load directly, while the math runs on our ops:
fused QKV projection, the gfx950 flash-attention kernel (causal, head_dim 64/128) or the fp32
reference, LayerNorm / GELU kernels.

Notebook variants (``Transformer/Transformer_Advanced.ipynb`` cells 4-24): MHA, GQA, MQA,
MLA with decoupled RoPE (returns the latent KV cache), LocalAttention (sliding window — a
banded mask instead of the notebook's per-query Python loop), ResiDual / Parallel blocks,
StochasticDepth and MoE feed-forward (dense "compute every expert" and sparse dispatch).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import reference as ref
from ..ops.activation import gelu
from ..ops.attention import sdpa_bshd
from ..ops.moe import moe_combine, moe_dispatch, moe_gather, moe_route
from ..ops.norm import LayerNorm


def sinusoidal_pe(n: int, d: int) -> torch.Tensor:
    """Fixed sin/cos table [n, d] (``ddp_gpt_wikitext2.py:134-139``)."""
    pe = torch.zeros(n, d)
    pos = torch.arange(0, n, dtype=torch.float).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2).float() * (-math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe


def _mask_kind(attn_mask, L: int):
    """Recognise the reference's causal masks (bool triu or -inf triu) → 'causal'."""
    if attn_mask is None:
        return None, None
    if attn_mask.dim() == 2 and attn_mask.shape == (L, L):
        tri = torch.ones(L, L, dtype=torch.bool, device=attn_mask.device).triu(1)
        m = attn_mask if attn_mask.dtype == torch.bool else torch.isinf(attn_mask) & (attn_mask < 0)
        if torch.equal(m, tri):
            return "causal", None
    return "explicit", attn_mask


class MultiheadAttention(nn.Module):
    """``nn.MultiheadAttention``-compatible self/cross attention."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, bias=True, batch_first=False, device=None, dtype=None):
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout, self.batch_first = embed_dim, num_heads, dropout, batch_first
        self.head_dim = embed_dim // num_heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim, device=device, dtype=dtype))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * embed_dim, device=device, dtype=dtype)) if bias else None
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias, device=device, dtype=dtype)
        nn.init.xavier_uniform_(self.in_proj_weight)
        if bias:
            nn.init.zeros_(self.out_proj.bias)

    def forward(self, query, key=None, value=None, attn_mask=None, key_padding_mask=None, need_weights=False,
                is_causal=False):
        key = query if key is None else key
        value = key if value is None else value
        if not self.batch_first:      # [L, N, E] layout (the nn default the minigpt reference relies on)
            query, key, value = (t.transpose(0, 1) for t in (query, key, value))
        B, L, E = query.shape
        H, D = self.num_heads, self.head_dim
        w, b = self.in_proj_weight, self.in_proj_bias
        if query is key and key is value:
            qkv = F.linear(query, w, b)
            q, k, v = qkv.split(E, dim=-1)
        else:
            q = F.linear(query, w[:E], None if b is None else b[:E])
            k = F.linear(key, w[E:2 * E], None if b is None else b[E:2 * E])
            v = F.linear(value, w[2 * E:], None if b is None else b[2 * E:])
        S = k.shape[1]
        q, k, v = q.reshape(B, L, H, D), k.reshape(B, S, H, D), v.reshape(B, S, H, D)
        kind, m = _mask_kind(attn_mask, L)
        causal = is_causal or kind == "causal"
        drop = self.dropout if self.training else 0.0
        if kind == "explicit" or (key_padding_mask is not None and key_padding_mask.dtype != torch.bool):
            o = _explicit_attention(q, k, v, m, key_padding_mask, drop)
        else:
            kpm = None if key_padding_mask is None else ~key_padding_mask   # nn: True = ignore
            o = sdpa_bshd(q, k, v, causal=causal, dropout_p=drop, key_padding_mask=kpm)
        o = self.out_proj(o.reshape(B, L, E))
        if not self.batch_first:
            o = o.transpose(0, 1)
        return o, None


def _explicit_attention(q, k, v, mask, key_padding_mask, dropout_p):
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if mask is not None:
        s = s.masked_fill(mask, float("-inf")) if mask.dtype == torch.bool else s + mask.float()
    if key_padding_mask is not None:
        s = s.masked_fill(key_padding_mask[:, None, None, :].bool(), float("-inf"))
    p = torch.nan_to_num(torch.softmax(s, -1))
    if dropout_p > 0:
        p = F.dropout(p, dropout_p)
    return (p @ vf).transpose(1, 2).to(q.dtype)


def _act(name):
    return {"relu": F.relu, "gelu": gelu}[name] if isinstance(name, str) else name


class TransformerEncoderLayer(nn.Module):
    """``nn.TransformerEncoderLayer`` semantics (post-LN by default)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu",
                 layer_norm_eps=1e-5, batch_first=False, norm_first=False):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, nhead, dropout, batch_first=batch_first)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm_first = norm_first
        self.norm1 = LayerNorm(d_model, eps=layer_norm_eps)
        self.norm2 = LayerNorm(d_model, eps=layer_norm_eps)
        self.dropout1, self.dropout2 = nn.Dropout(dropout), nn.Dropout(dropout)
        self.activation = _act(activation)

    def _sa(self, x, mask, kpm, is_causal):
        return self.dropout1(self.self_attn(x, x, x, attn_mask=mask, key_padding_mask=kpm, is_causal=is_causal)[0])

    def _ff(self, x):
        return self.dropout2(self.linear2(self.dropout(self.activation(self.linear1(x)))))

    def forward(self, src, src_mask=None, src_key_padding_mask=None, is_causal=False):
        x = src
        if self.norm_first:
            x = x + self._sa(self.norm1(x), src_mask, src_key_padding_mask, is_causal)
            return x + self._ff(self.norm2(x))
        x = self.norm1(x + self._sa(x, src_mask, src_key_padding_mask, is_causal))
        return self.norm2(x + self._ff(x))


class TransformerEncoder(nn.Module):
    def __init__(self, encoder_layer: TransformerEncoderLayer, num_layers: int, make_layer=None):
        super().__init__()
        self.layers = nn.ModuleList([make_layer() if make_layer else encoder_layer for _ in range(num_layers)])

    def forward(self, src, mask=None, src_key_padding_mask=None, is_causal=False):
        for layer in self.layers:
            src = layer(src, mask, src_key_padding_mask, is_causal)
        return src


class TransformerDecoderLayer(nn.Module):
    """``nn.TransformerDecoderLayer`` semantics: self-attn, cross-attn to ``memory``, FFN."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu",
                 layer_norm_eps=1e-5, batch_first=False, norm_first=False):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, nhead, dropout, batch_first=batch_first)
        self.multihead_attn = MultiheadAttention(d_model, nhead, dropout, batch_first=batch_first)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.dropout = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm_first = norm_first
        self.norm1 = LayerNorm(d_model, eps=layer_norm_eps)
        self.norm2 = LayerNorm(d_model, eps=layer_norm_eps)
        self.norm3 = LayerNorm(d_model, eps=layer_norm_eps)
        self.dropout1, self.dropout2, self.dropout3 = nn.Dropout(dropout), nn.Dropout(dropout), nn.Dropout(dropout)
        self.activation = _act(activation)

    def _cross(self, x, memory, memory_is_zero: bool):
        if memory_is_zero:
            # K = b_k, V = b_v for every memory slot → uniform attention; output = out_proj(b_v)
            # exactly (the reference feeds a zero "memory", minigpt/model.py:19,28-30)
            E = x.shape[-1]
            bv = self.multihead_attn.in_proj_bias[2 * E:] if self.multihead_attn.in_proj_bias is not None \
                else x.new_zeros(E)
            return self.multihead_attn.out_proj(bv).expand_as(x)
        return self.multihead_attn(x, memory, memory)[0]

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, tgt_key_padding_mask=None,
                memory_key_padding_mask=None, tgt_is_causal=False, memory_is_causal=False, memory_is_zero=False):
        x = tgt
        sa = lambda t: self.self_attn(t, t, t, attn_mask=tgt_mask, key_padding_mask=tgt_key_padding_mask,  # noqa
                                      is_causal=tgt_is_causal)[0]
        ff = lambda t: self.linear2(self.dropout(self.activation(self.linear1(t))))  # noqa
        if self.norm_first:
            x = x + self.dropout1(sa(self.norm1(x)))
            x = x + self.dropout2(self._cross(self.norm2(x), memory, memory_is_zero))
            return x + self.dropout3(ff(self.norm3(x)))
        x = self.norm1(x + self.dropout1(sa(x)))
        x = self.norm2(x + self.dropout2(self._cross(x, memory, memory_is_zero)))
        return self.norm3(x + self.dropout3(ff(x)))


# ============================================================================ notebook variants
class _HeadsAttention(nn.Module):
    """Shared core: Q from W_q, K/V with ``kv_heads`` heads, causal or windowed."""

    def __init__(self, d_model, num_heads, kv_heads, window: int | None = None, causal: bool = False):
        super().__init__()
        assert d_model % num_heads == 0 and num_heads % kv_heads == 0
        self.d_model, self.num_heads, self.kv_heads = d_model, num_heads, kv_heads
        self.d_head = d_model // num_heads
        self.W_q = nn.Linear(d_model, d_model)
        self.W_k = nn.Linear(d_model, self.d_head * kv_heads)
        self.W_v = nn.Linear(d_model, self.d_head * kv_heads)
        self.W_o = nn.Linear(d_model, d_model)
        self.window, self.causal = window, causal

    def forward(self, x, mask=None):
        B, L, _ = x.shape
        q = self.W_q(x).view(B, L, self.num_heads, self.d_head)
        k = self.W_k(x).view(B, L, self.kv_heads, self.d_head)
        v = self.W_v(x).view(B, L, self.kv_heads, self.d_head)
        if mask is not None:
            rep = self.num_heads // self.kv_heads
            o = _explicit_attention(q, k.repeat_interleave(rep, 2), v.repeat_interleave(rep, 2),
                                    mask == 0 if mask.dtype != torch.bool else ~mask, None, 0.0)
        elif self.window is not None:
            o = _window_attention(q, k, v, self.window)
        else:
            o = sdpa_bshd(q, k, v, causal=self.causal)
        return self.W_o(o.reshape(B, L, self.d_model))


def _window_attention(q, k, v, w):
    """Symmetric sliding window |i-j| <= w (the notebook's LocalAttention, cell 12)."""
    B, L, H, D = q.shape
    rep = H // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().repeat_interleave(rep, 2).transpose(1, 2)
    vf = v.float().repeat_interleave(rep, 2).transpose(1, 2)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    i = torch.arange(L, device=q.device)
    s = s.masked_fill((i[:, None] - i[None, :]).abs() > w, float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2).to(q.dtype)


class MultiHeadAttention(_HeadsAttention):
    def __init__(self, d_model, num_heads, causal=False):
        super().__init__(d_model, num_heads, num_heads, causal=causal)


class GroupedQueryAttention(_HeadsAttention):
    """GQA: ``num_groups`` K/V heads shared by ``num_heads / num_groups`` query heads (cell 6)."""

    def __init__(self, d_model, num_heads, num_groups, causal=False):
        super().__init__(d_model, num_heads, num_groups, causal=causal)


class MultiQueryAttention(_HeadsAttention):
    """MQA: a single K/V head (cell 8)."""

    def __init__(self, d_model, num_heads, causal=False):
        super().__init__(d_model, num_heads, 1, causal=causal)


class LocalAttention(_HeadsAttention):
    """Sliding-window attention, window ±``window_size`` (cell 12)."""

    def __init__(self, d_model, num_heads, window_size):
        super().__init__(d_model, num_heads, num_heads, window=window_size)


class MultiHeadLatentAttention(nn.Module):
    """MLA with a shared KV down-projection and decoupled RoPE on the last ``d_rope`` latent
    dims (rotate-half); returns (output, latent KV cache C_kv) like the notebook (cell 10)."""

    def __init__(self, d_model, num_heads, d_latent, d_rope=64, causal=False, theta=10000.0):
        super().__init__()
        assert d_model % num_heads == 0 and d_latent >= d_rope and d_rope % 2 == 0
        self.d_model, self.num_heads, self.d_head = d_model, num_heads, d_model // num_heads
        self.d_latent, self.d_rope, self.d_nope = d_latent, d_rope, d_latent - d_rope
        self.W_dkv = nn.Linear(d_model, d_latent)
        self.W_dq = nn.Linear(d_model, d_latent)
        self.W_uq = nn.Linear(d_latent, d_model)
        self.W_uk = nn.Linear(d_latent, d_model)
        self.W_uv = nn.Linear(d_latent, d_model)
        self.W_o = nn.Linear(d_model, d_model)
        half = d_rope // 2
        self.register_buffer("freqs", 1.0 / (theta ** (torch.arange(0, half).float() / half)), persistent=False)
        self.causal = causal

    def apply_decoupled_rope(self, x, positions):
        ang = positions[:, None].float() * self.freqs[None, :]
        c, s = torch.cos(ang), torch.sin(ang)
        x_nope, x_rope = x[..., :self.d_nope], x[..., self.d_nope:]
        h = self.d_rope // 2
        x1, x2 = x_rope[..., :h], x_rope[..., h:]
        return torch.cat([x_nope, x1 * c - x2 * s, x1 * s + x2 * c], -1)

    def forward(self, x, positions=None):
        B, L, _ = x.shape
        pos = torch.arange(L, device=x.device) if positions is None else positions
        c_kv = self.apply_decoupled_rope(self.W_dkv(x), pos)
        c_q = self.apply_decoupled_rope(self.W_dq(x), pos)
        q = self.W_uq(c_q).view(B, L, self.num_heads, self.d_head)
        k = self.W_uk(c_kv).view(B, L, self.num_heads, self.d_head)
        v = self.W_uv(c_kv).view(B, L, self.num_heads, self.d_head)
        o = sdpa_bshd(q, k, v, causal=self.causal)
        return self.W_o(o.reshape(B, L, self.d_model)), c_kv


def _ffn(d_model, d_ff, dropout, act="gelu"):
    return nn.Sequential(nn.Linear(d_model, d_ff), nn.GELU() if act == "gelu" else nn.ReLU(),
                         nn.Linear(d_ff, d_model), nn.Dropout(dropout))


class ResiDualTransformerBlock(nn.Module):
    """Triple-LN "ResiDual" block (cell 17): y = x + LN3(y1 + FFN(LN2(y1))), y1 = LN1(x) + Attn."""

    def __init__(self, d_model, n_heads, d_ff, dropout=0.1):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, n_heads, dropout=dropout, batch_first=True)
        self.ffn = _ffn(d_model, d_ff, dropout)
        self.ln1, self.ln2, self.ln3 = LayerNorm(d_model), LayerNorm(d_model), LayerNorm(d_model)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, attn_mask=None):
        x_ln = self.ln1(x)
        y1 = x_ln + self.dropout(self.self_attn(x_ln, x_ln, x_ln, attn_mask=attn_mask)[0])
        y2 = y1 + self.ffn(self.ln2(y1))
        return x + self.ln3(y2)


class ParallelTransformerBlock(nn.Module):
    """Attention and FFN branches in parallel off one LayerNorm (cell 19)."""

    def __init__(self, d_model, n_heads, d_ff, dropout=0.1):
        super().__init__()
        self.ln = LayerNorm(d_model)
        self.self_attn = MultiheadAttention(d_model, n_heads, dropout=dropout, batch_first=True)
        self.ffn = _ffn(d_model, d_ff, dropout)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, attn_mask=None):
        x_ln = self.ln(x)
        a = self.dropout(self.self_attn(x_ln, x_ln, x_ln, attn_mask=attn_mask)[0])
        f = self.dropout(self.ffn(x_ln))
        return x + self.dropout(x_ln + a + f)


class StochasticDepth(nn.Module):
    """Per-sample residual-branch drop with 1/keep rescaling (cell 21)."""

    def __init__(self, drop_prob: float):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x, residual):
        if not self.training or self.drop_prob == 0.0:
            return x + residual
        keep = 1 - self.drop_prob
        mask = torch.empty(x.shape[0], *([1] * (x.dim() - 1)), device=x.device, dtype=x.dtype).bernoulli_(keep)
        return x + residual / keep * mask


class StochasticDepthBlock(nn.Module):
    def __init__(self, d_model, nhead, dim_ff, drop_prob=0.1):
        super().__init__()
        self.ln1, self.ln2 = LayerNorm(d_model), LayerNorm(d_model)
        self.attn = MultiheadAttention(d_model, nhead, batch_first=True)
        self.ffn = nn.Sequential(nn.Linear(d_model, dim_ff), nn.ReLU(), nn.Linear(dim_ff, d_model))
        self.sd1, self.sd2 = StochasticDepth(drop_prob), StochasticDepth(drop_prob)

    def forward(self, x):
        h = self.ln1(x)
        x = self.sd1(x, self.attn(h, h, h)[0])
        return self.sd2(x, self.ffn(self.ln2(x)))


class Expert(nn.Module):
    def __init__(self, d_model, hidden, dropout=0.0, act="gelu"):
        super().__init__()
        self.net = _ffn(d_model, hidden, dropout, act)

    def forward(self, x):
        return self.net(x)


class MoEFeedForward(nn.Module):
    """Top-k routed experts + optional shared experts.

    ``routing``: ``"topk_softmax"`` (DeepSeekLike: top-k over raw router logits, softmax over
    the k values, ``DeepSeekLike_wikitext2.py:276-309``) or ``"softmax_topk"`` (notebook cell
    24: softmax over all experts, then top-k of the probabilities, unnormalised).
    ``dispatch``: ``"sparse"`` — tokens are sorted by expert, each expert runs once on its
    contiguous slice, outputs are gate-weighted and scatter-added (index_add) — or
    ``"dense"`` (every expert on every token, masked; the notebook's formulation).
    """

    def __init__(self, d_model, hidden, num_experts=8, top_k=2, num_shared=0, dropout=0.0,
                 routing="topk_softmax", dispatch="sparse", act="gelu"):
        super().__init__()
        self.num_experts, self.top_k, self.num_shared = num_experts, top_k, num_shared
        self.router = nn.Linear(d_model, num_experts)
        self.experts = nn.ModuleList([Expert(d_model, hidden, dropout, act) for _ in range(num_experts)])
        self.shared_experts = nn.ModuleList([Expert(d_model, hidden, dropout, act) for _ in range(num_shared)])
        self.dropout = nn.Dropout(dropout)
        self.routing, self.dispatch = routing, dispatch
        self.last_router_probs = None

    @property
    def gate(self):  # notebook name
        return self.router

    def route(self, x_flat):
        logits = self.router(x_flat)
        k = min(self.top_k, self.num_experts)
        w, idx = moe_route(logits, k, self.routing)
        self.last_router_probs = F.softmax(logits.float(), -1)
        return w, idx

    def forward(self, x):
        shape = x.shape
        xf = x.reshape(-1, shape[-1])
        shared = None
        if self.num_shared:
            shared = sum(e(xf) for e in self.shared_experts) / self.num_shared
        w, idx = self.route(xf)
        if self.dispatch == "dense":
            out = torch.zeros_like(xf) if shared is None else shared
            for j in range(idx.shape[1]):
                eo = torch.zeros_like(xf)
                for e, expert in enumerate(self.experts):
                    m = (idx[:, j] == e).unsqueeze(-1).to(xf.dtype)
                    eo = eo + m * expert(xf)
                out = out + eo * w[:, j:j + 1].to(xf.dtype)
        else:
            # expert-sorted dispatch (ops/moe.py: HIP routing/permute/gather/combine kernels);
            # one host read of the segment offsets drives the per-expert GEMMs
            d = moe_dispatch(idx, self.num_experts)
            xs = moe_gather(xf, d)
            ys, s = [], 0
            for e, c in enumerate(d.counts()):
                if c:
                    ys.append(self.experts[e](xs[s:s + c]))
                s += c
            y = torch.cat(ys, 0) if ys else xs
            out = moe_combine(y, d, w, shared)
        return self.dropout(out.view(shape))


def load_balance_loss(router_probs: torch.Tensor, idx: torch.Tensor, num_experts: int) -> torch.Tensor:
    """Switch-style auxiliary loss (fraction routed × mean prob), optional for MoE training."""
    frac = torch.bincount(idx.reshape(-1), minlength=num_experts).float() / idx.numel()
    return num_experts * (frac * router_probs.mean(0)).sum()
