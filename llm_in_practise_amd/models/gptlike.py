"""GPT-like pretraining models of the distributed-training tracks.

``GPTLike`` — pre-LN blocks ``x + attn(ln1(x))``, ``x + mlp(ln2(x))`` with ``nn.MultiheadAttention``
(causal), GELU 4× MLP, tied head, and one of:
  * ``pos="sinusoidal"``: fixed table registered as ``pos_emb`` buffer [1, block, d]
    (``ddp_gpt_wikitext2.py:134-139``, ``GPTLike_wikitext2_fixed_pe.py``);
  * ``pos="learned"``: ``pos_emb = Embedding(block, d)`` (``GPTLike_wikitext2_learned_pe.py:166``,
    ``temp/ddp_gpt_wikitext2.py:176``).
``init="xavier"`` is the C/D family (``ddp_gpt_wikitext2.py:147-155``), ``init="normal"`` the
B family / temp scripts (N(0, 0.02)).  State-dict keys are the reference's, so
``models/final_model.pth`` / per-epoch checkpoints load directly.

``SimpleTransformer`` — B1 (``GPTLike_wikitext2.py:95-138``): encoder stack with fixed PE and no
causal mask (kept as in the reference; ``causal=True`` opt-in).

Named presets: ``gptlike-bert`` (C1-C3/D1-D4: 6 layers, d768, 12 heads, vocab 30522),
``gptlike-multihost`` (D5: 12 layers, d1024, 16 heads, vocab 50258, block 512),
``gpt-byte`` (C4: vocab 256, d512, 8 heads, learned PE), ``gptlike-bpe`` (B2: vocab 30000, d768, 8 heads).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.loss import fused_linear_cross_entropy
from ..ops.norm import LayerNorm
from ..ops.embedding import Embedding
from .layers import MultiheadAttention, TransformerEncoderLayer, sinusoidal_pe


class CausalSelfAttention(nn.Module):
    def __init__(self, d_model, n_head, dropout=0.1, attn_dropout=None):
        super().__init__()
        self.mha = MultiheadAttention(d_model, n_head, dropout=dropout if attn_dropout is None else attn_dropout,
                                      batch_first=True)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        return self.dropout(self.mha(x, x, x, is_causal=True)[0])


class FeedForward(nn.Module):
    def __init__(self, d_model, hidden_dim, dropout=0.1):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(d_model, hidden_dim), nn.GELU(), nn.Linear(hidden_dim, d_model),
                                 nn.Dropout(dropout))

    def forward(self, x):
        return self.net(x)


class TransformerBlock(nn.Module):
    def __init__(self, d_model, n_head, dropout=0.1, mlp_ratio=4.0, attn_dropout=None):
        super().__init__()
        self.ln1 = LayerNorm(d_model)
        self.attn = CausalSelfAttention(d_model, n_head, dropout, attn_dropout)
        self.ln2 = LayerNorm(d_model)
        self.mlp = FeedForward(d_model, int(d_model * mlp_ratio), dropout)

    def forward(self, x):
        x = x + self.attn(self.ln1(x))
        return x + self.mlp(self.ln2(x))


PRESETS = {
    "gptlike-bert": dict(vocab_size=30522, block_size=512, n_layer=6, n_head=12, d_model=768),
    "gptlike-multihost": dict(vocab_size=50258, block_size=512, n_layer=12, n_head=16, d_model=1024),
    "gptlike-bpe": dict(vocab_size=30000, block_size=256, n_layer=6, n_head=8, d_model=768, init="normal"),
    "gpt-byte": dict(vocab_size=256, block_size=128, n_layer=6, n_head=8, d_model=512, pos="learned",
                     init="normal"),
    "gptlike-tiny": dict(vocab_size=512, block_size=64, n_layer=2, n_head=4, d_model=64),
}


class GPTLike(nn.Module):
    def __init__(self, vocab_size=30522, block_size=256, n_layer=6, n_head=12, d_model=768, dropout=0.1,
                 pos: str = "sinusoidal", init: str = "xavier", tie: bool = True):
        super().__init__()
        self.config = dict(vocab_size=vocab_size, block_size=block_size, n_layer=n_layer, n_head=n_head,
                           d_model=d_model, dropout=dropout, pos=pos, init=init, tie=tie)
        self.tok_emb = Embedding(vocab_size, d_model)
        self.drop = nn.Dropout(dropout)
        self.blocks = nn.ModuleList([TransformerBlock(d_model, n_head, dropout) for _ in range(n_layer)])
        self.ln_f = LayerNorm(d_model)
        self.head = nn.Linear(d_model, vocab_size, bias=False)
        if tie:
            self.head.weight = self.tok_emb.weight
        self.block_size, self.d_model, self.pos = block_size, d_model, pos
        if pos == "learned":
            self.pos_emb = Embedding(block_size, d_model)
        else:
            self.register_buffer("pos_emb", sinusoidal_pe(block_size, d_model).unsqueeze(0), persistent=True)
        self.init = init
        self.apply(self._init_weights)

    @classmethod
    def from_preset(cls, name: str, **kw):
        cfg = dict(PRESETS[name])
        cfg.update(kw)
        return cls(**cfg)

    def _init_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            if self.init == "xavier":
                nn.init.xavier_uniform_(module.weight)
            else:
                nn.init.normal_(module.weight, mean=0.0, std=0.02)
        if isinstance(module, nn.Linear) and module.bias is not None:
            nn.init.zeros_(module.bias)
        if isinstance(module, nn.LayerNorm):
            nn.init.zeros_(module.bias)
            nn.init.ones_(module.weight)

    def resize_token_embeddings(self, n: int):
        """Grow/shrink the vocabulary keeping the tie (``temp/ddp_gpt_bpe_tokenizer.py:215-247``)."""
        old = self.tok_emb
        new = Embedding(n, self.d_model, device=old.weight.device, dtype=old.weight.dtype)
        nn.init.normal_(new.weight, 0.0, 0.02)
        k = min(n, old.num_embeddings)
        with torch.no_grad():
            new.weight[:k] = old.weight[:k]
        self.tok_emb = new
        self.head = nn.Linear(self.d_model, n, bias=False, device=new.weight.device, dtype=new.weight.dtype)
        self.head.weight = self.tok_emb.weight
        self.config["vocab_size"] = n
        return self

    def hidden(self, idx):
        B, L = idx.shape
        if L > self.block_size:
            idx = idx[:, :self.block_size]
            L = self.block_size
        if self.pos == "learned":
            x = self.tok_emb(idx) + self.pos_emb(torch.arange(L, device=idx.device))[None]
        else:
            x = self.tok_emb(idx) + self.pos_emb[:, :L, :].to(self.tok_emb.weight.dtype)
        x = self.drop(x)
        for blk in self.blocks:
            x = blk(x)
        return self.ln_f(x)

    def forward(self, idx, targets=None):
        """Returns logits [B, L, V]; with ``targets`` returns (logits=None, loss) computed by the
        chunked LM-head + cross-entropy kernel (no [B·L, V] fp32 logits)."""
        h = self.hidden(idx)
        if targets is None:
            return self.head(h)
        loss = fused_linear_cross_entropy(h.reshape(-1, h.shape[-1]), self.head.weight, targets.reshape(-1))
        return None, loss

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())


class SimpleTransformer(nn.Module):
    """B1 ``SimpleTransformer`` (encoder stack, fixed PE; the reference passes no causal mask)."""

    def __init__(self, vocab_size, d_model=256, nhead=4, num_layers=6, max_len=64, dropout=0.1, causal=False):
        super().__init__()
        self.d_model, self.max_len, self.causal = d_model, max_len, causal
        self.token_embedding = Embedding(vocab_size, d_model)
        self.register_buffer("pos_embedding", sinusoidal_pe(max_len, d_model).unsqueeze(0))
        self.transformer = _Stack(d_model, nhead, num_layers, dropout)
        self.output_layer = nn.Linear(d_model, vocab_size)

    def forward(self, x):
        h = self.token_embedding(x) + self.pos_embedding[:, :x.size(1), :]
        return self.output_layer(self.transformer(h, self.causal))


class _Stack(nn.Module):
    def __init__(self, d, h, n, dropout):
        super().__init__()
        self.layers = nn.ModuleList([TransformerEncoderLayer(d, h, 4 * d, dropout, activation="gelu",
                                                             batch_first=True) for _ in range(n)])

    def forward(self, x, causal=False):
        for layer in self.layers:
            x = layer(x, is_causal=causal)
        return x
