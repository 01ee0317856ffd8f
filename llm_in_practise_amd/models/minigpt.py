"""llm-demo MiniGPT models.

``MiniGPT``   — ``llm-demo/minigpt/model.py:5-32``: token + learned positional embedding (16
                positions), a stack of decoder layers fed a zero "memory", linear head.  The
                reference passes ``[batch, seq, E]`` into ``nn.TransformerDecoderLayer`` whose
                default layout is ``[seq, batch, E]`` and gives no causal mask, so attention
                actually runs across the batch dimension.  ``reference_layout=True`` (default)
                reproduces that exactly — reference checkpoints load and behave identically;
                ``reference_layout=False, causal=True`` is the corrected causal char-LM.
``MiniGPT2``  — ``llm-demo/minigpt2/model.py:39-72``: encoder-only (GELU, 4× FFN, batch_first),
                ``nn.Parameter`` positional table, final LayerNorm, N(0, 0.02) init, no mask by
                default (``causal=True`` opt-in).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn

from ..ops.norm import LayerNorm
from ..ops.embedding import Embedding
from .layers import TransformerDecoderLayer, TransformerEncoderLayer


class MiniGPT(nn.Module):
    def __init__(self, vocab_size, embed_dim=64, n_heads=2, n_layers=2, dropout=0.1, seq_len=16,
                 reference_layout: bool = True, causal: bool = False, dim_feedforward: int = 2048):
        super().__init__()
        self.token_embed = Embedding(vocab_size, embed_dim)
        self.pos_embed = Embedding(seq_len, embed_dim)
        self.layers = nn.ModuleList([
            TransformerDecoderLayer(embed_dim, n_heads, dim_feedforward, dropout, batch_first=not reference_layout)
            for _ in range(n_layers)])
        self.register_buffer("dummy_memory", torch.zeros(1, 1, embed_dim))
        self.fc = nn.Linear(embed_dim, vocab_size)
        self.reference_layout, self.causal = reference_layout, causal

    def forward(self, x):
        pos = torch.arange(0, x.size(1), dtype=torch.long, device=x.device)
        h = self.token_embed(x) + self.pos_embed(pos)
        B, S = x.shape
        memory = self.dummy_memory.expand(B, S, -1)
        for layer in self.layers:
            h = layer(h, memory, tgt_is_causal=self.causal and not self.reference_layout, memory_is_zero=True)
        return self.fc(h)


@dataclasses.dataclass
class MiniGPT2Config:
    """Mirror of the reference's class-attribute ``Config`` (``minigpt2/model.py:4-13``)."""
    seq_len: int = 256
    n_layer: int = 4
    n_head: int = 4
    embed_dim: int = 128
    dropout: float = 0.1
    lr: float = 3e-4
    weight_decay: float = 0.1
    epochs: int = 200
    batch_size: int = 2
    vocab_size: int = 0

    @classmethod
    def from_dict(cls, d):
        f = {x.name for x in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in f})


class MiniGPT2(nn.Module):
    def __init__(self, config: MiniGPT2Config, causal: bool = False):
        super().__init__()
        c = config
        self.config, self.causal = c, causal
        self.embed = Embedding(c.vocab_size, c.embed_dim)
        self.pos_embed = nn.Parameter(torch.zeros(1, c.seq_len, c.embed_dim))
        self.transformer = _Encoder(c)
        self.ln = LayerNorm(c.embed_dim)
        self.head = nn.Linear(c.embed_dim, c.vocab_size)
        self.apply(self._init_weights)

    @staticmethod
    def _init_weights(module):
        if isinstance(module, nn.Linear):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                nn.init.zeros_(module.bias)

    def forward(self, x):
        T = x.shape[1]
        h = self.embed(x) + self.pos_embed[:, :T, :]
        h = self.transformer(h, is_causal=self.causal)
        return self.head(self.ln(h))


class _Encoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layers = nn.ModuleList([
            TransformerEncoderLayer(c.embed_dim, c.n_head, 4 * c.embed_dim, c.dropout, activation="gelu",
                                    batch_first=True) for _ in range(c.n_layer)])

    def forward(self, x, is_causal=False):
        for layer in self.layers:
            x = layer(x, is_causal=is_causal)
        return x
