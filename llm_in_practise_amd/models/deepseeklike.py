"""DeepSeek-like model: causal MLA + MoE FFN + RoPE.

``CausalMLA`` (``DeepSeekLike_wikitext2.py:168-238``): full-rank q/k/v projections, RoPE on
q/k (interleaved pairs — the complex-multiply form — or the even/odd cos/sin form of B6, both
the same rotation), per-head linear compression head_dim → latent (default head_dim/4) of
q, k, v, causal attention at scale 1/√latent, decompression latent → head_dim, out_proj.
RoPE runs on the ``rope`` HIP kernel (interleaved layout) on the GPU.

``MoEFeedForward``: router → top-k over raw logits → softmax over the k → experts; shared
experts averaged.  ``moe_dispatch="dense"`` is B5's masked loop, ``"sparse"`` B6's
gather / index_add (sort-by-expert on our side).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..ops import reference as ref
from ..ops.attention import sdpa_bshd
from ..ops.loss import fused_linear_cross_entropy
from ..ops.norm import LayerNorm
from ..ops.rope import apply_rope
from ..ops.embedding import Embedding
from .layers import MoEFeedForward


class CausalMLA(nn.Module):
    def __init__(self, embed_dim, num_heads, latent_dim=None, attn_dropout=0.0, resid_dropout=0.0):
        super().__init__()
        assert embed_dim % num_heads == 0
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        assert self.head_dim % 2 == 0, "head_dim must be even for RoPE"
        self.latent_dim = max(1, latent_dim if latent_dim is not None else max(1, self.head_dim // 4))
        self.q_proj = nn.Linear(embed_dim, embed_dim)
        self.k_proj = nn.Linear(embed_dim, embed_dim)
        self.v_proj = nn.Linear(embed_dim, embed_dim)
        self.q_compress = nn.Linear(self.head_dim, self.latent_dim)
        self.k_compress = nn.Linear(self.head_dim, self.latent_dim)
        self.v_compress = nn.Linear(self.head_dim, self.latent_dim)
        self.decompress = nn.Linear(self.latent_dim, self.head_dim)
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        self.dropout = nn.Dropout(resid_dropout)
        self.attn_dropout = attn_dropout

    def forward(self, x, cos, sin):
        B, L, D = x.shape
        H, hd = self.num_heads, self.head_dim
        q = self.q_proj(x).view(B, L, H, hd)
        k = self.k_proj(x).view(B, L, H, hd)
        v = self.v_proj(x).view(B, L, H, hd)
        q = apply_rope(q.reshape(B * L, H, hd).contiguous(), cos, sin, interleaved=True).view(B, L, H, hd)
        k = apply_rope(k.reshape(B * L, H, hd).contiguous(), cos, sin, interleaved=True).view(B, L, H, hd)
        qc, kc, vc = self.q_compress(q), self.k_compress(k), self.v_compress(v)
        o = sdpa_bshd(qc, kc, vc, causal=True, scale=1.0 / math.sqrt(max(1, self.latent_dim)),
                      dropout_p=self.attn_dropout if self.training else 0.0)
        o = self.decompress(o).reshape(B, L, D)
        return self.dropout(self.out_proj(o))


class TransformerBlock(nn.Module):
    def __init__(self, d_model, nhead, mlp_ratio=4.0, dropout=0.1, latent_dim=None, num_experts=8, top_k=2,
                 num_shared=2, moe_dispatch="sparse"):
        super().__init__()
        self.ln1 = LayerNorm(d_model)
        self.attn = CausalMLA(d_model, nhead, latent_dim=latent_dim, attn_dropout=0.0, resid_dropout=dropout)
        self.ln2 = LayerNorm(d_model)
        self.mlp = MoEFeedForward(d_model, int(d_model * mlp_ratio), num_experts, top_k, num_shared, dropout,
                                  routing="topk_softmax", dispatch=moe_dispatch)

    def forward(self, x, cos, sin):
        x = x + self.attn(self.ln1(x), cos, sin)
        return x + self.mlp(self.ln2(x))


class DeepSeekLike(nn.Module):
    def __init__(self, vocab_size=30000, block_size=256, n_layer=6, n_head=8, d_model=768, dropout=0.1,
                 latent_dim=None, num_experts=8, top_k=2, num_shared=2, rope_theta=10000.0, moe_dispatch="sparse"):
        super().__init__()
        self.tok_emb = Embedding(vocab_size, d_model)
        self.drop = nn.Dropout(dropout)
        self.blocks = nn.ModuleList([
            TransformerBlock(d_model, n_head, 4.0, dropout, latent_dim, num_experts, top_k, num_shared, moe_dispatch)
            for _ in range(n_layer)])
        self.ln_f = LayerNorm(d_model)
        self.head = nn.Linear(d_model, vocab_size, bias=False)
        self.head.weight = self.tok_emb.weight
        self.block_size, self.d_model, self.n_head, self.rope_theta = block_size, d_model, n_head, rope_theta
        self.apply(self._init_weights)
        inv, _ = ref.rope_inv_freq(d_model // n_head, rope_theta)
        self.register_buffer("inv_freq", inv, persistent=False)

    @staticmethod
    def _init_weights(module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
        if isinstance(module, nn.Linear) and getattr(module, "bias", None) is not None:
            nn.init.zeros_(module.bias)

    def hidden(self, idx):
        B, L = idx.shape
        if L > self.block_size:
            idx = idx[:, :self.block_size]
            L = self.block_size
        ang = torch.arange(L, device=idx.device).float()[:, None] * self.inv_freq[None, :]
        cos = torch.cos(ang).repeat(B, 1).contiguous()
        sin = torch.sin(ang).repeat(B, 1).contiguous()
        x = self.drop(self.tok_emb(idx))
        for blk in self.blocks:
            x = blk(x, cos, sin)
        return self.ln_f(x)

    def forward(self, idx, targets=None):
        h = self.hidden(idx)
        if targets is None:
            return self.head(h)
        return None, fused_linear_cross_entropy(h.reshape(-1, h.shape[-1]), self.head.weight, targets.reshape(-1))
