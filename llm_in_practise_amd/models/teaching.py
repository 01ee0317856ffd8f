"""Transformer_Basics notebook models (``Transformer/Transformer_Basics.ipynb`` cells 20-41),
built on this package's attention / norm ops so they run the fused kernels on MI355X:

* :class:`Seq2SeqTransformer` — the full encoder-decoder Transformer of cell 22 (scaled
  embeddings, sinusoidal PE, post-LN encoder blocks, decoder blocks with masked self-attention +
  cross-attention to the encoder output, linear generator), with greedy ``translate``.
* :class:`DecoderOnlyTransformer` — cell 24 (decoder-only blocks under a triu mask).
* :class:`MiniBert` — cell 34's IMDb sentiment classifier: token + learned position embeddings,
  pre-LN encoder layers with a key-padding mask, final LayerNorm, ``[CLS]`` (position 0) pooling,
  linear classifier; trained with CrossEntropy / Adam(lr 1e-3, wd 1e-5), 2 epochs, batch 16,
  max_len 256 (driver: ``lipa minibert-imdb``).
* :class:`NotebookGPT` + :class:`NotebookGPTConfig` — cells 39 (WikiText-2, GPT-2 tokenizer,
  vocab 50257) and 41 (Chinese GPT on CLUECorpusSmall with the bert-base-chinese vocab 21128):
  n_embd 256, n_head 8, n_layer 6, triu-masked attention, multinomial ``generate``; AdamW(3e-4,
  wd 0.01) (driver: ``lipa nb-gpt``).
"""
from __future__ import annotations

import dataclasses
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.norm import LayerNorm
from ..ops.embedding import Embedding
from .layers import MultiheadAttention, sinusoidal_pe


class ScaledEmbedding(nn.Module):
    """cell 20/22 ``Embeddings``: lookup × √d_model."""

    def __init__(self, vocab_size: int, d_model: int):
        super().__init__()
        self.emb = Embedding(vocab_size, d_model)
        self.scale = math.sqrt(d_model)

    def forward(self, x):
        return self.emb(x) * self.scale


class _FF(nn.Module):
    def __init__(self, d_model, d_ff, dropout=0.0, act="relu"):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(d_model, d_ff), nn.Linear(d_ff, d_model)
        self.drop = nn.Dropout(dropout)
        self.act = F.gelu if act == "gelu" else F.relu

    def forward(self, x):
        return self.fc2(self.drop(self.act(self.fc1(x))))


class EncoderBlock(nn.Module):
    def __init__(self, d_model, num_heads, d_ff, dropout=0.0):
        super().__init__()
        self.attn = MultiheadAttention(d_model, num_heads, dropout, batch_first=True)
        self.ff = _FF(d_model, d_ff, dropout)
        self.ln1, self.ln2 = LayerNorm(d_model), LayerNorm(d_model)

    def forward(self, x, src_kpm=None):
        x = self.ln1(x + self.attn(x, key_padding_mask=src_kpm)[0])
        return self.ln2(x + self.ff(x))


class DecoderBlock(nn.Module):
    def __init__(self, d_model, num_heads, d_ff, dropout=0.0, cross: bool = True):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, num_heads, dropout, batch_first=True)
        self.cross_attn = MultiheadAttention(d_model, num_heads, dropout, batch_first=True) if cross else None
        self.ff = _FF(d_model, d_ff, dropout)
        self.ln1, self.ln3 = LayerNorm(d_model), LayerNorm(d_model)
        self.ln2 = LayerNorm(d_model) if cross else None

    def forward(self, x, memory=None, mem_kpm=None):
        x = self.ln1(x + self.self_attn(x, is_causal=True)[0])
        if self.cross_attn is not None:
            x = self.ln2(x + self.cross_attn(x, memory, memory, key_padding_mask=mem_kpm)[0])
        return self.ln3(x + self.ff(x))


class Seq2SeqTransformer(nn.Module):
    """cell 22 ``Transformer(src_vocab_size, tgt_vocab_size, d_model, num_heads, d_ff, num_layers=6)``."""

    def __init__(self, src_vocab_size: int, tgt_vocab_size: int, d_model: int = 64, num_heads: int = 4,
                 d_ff: int = 256, num_layers: int = 6, max_len: int = 5000, dropout: float = 0.0, pad_id: int = 0):
        super().__init__()
        self.src_emb, self.tgt_emb = ScaledEmbedding(src_vocab_size, d_model), ScaledEmbedding(tgt_vocab_size, d_model)
        self.register_buffer("pe", sinusoidal_pe(max_len, d_model), persistent=False)
        self.encoder = nn.ModuleList([EncoderBlock(d_model, num_heads, d_ff, dropout) for _ in range(num_layers)])
        self.decoder = nn.ModuleList([DecoderBlock(d_model, num_heads, d_ff, dropout) for _ in range(num_layers)])
        self.generator = nn.Linear(d_model, tgt_vocab_size)
        self.pad_id = pad_id

    def encode(self, src):
        kpm = src == self.pad_id                              # nn convention: True = ignore
        x = self.src_emb(src) + self.pe[:src.shape[1]].to(self.src_emb.emb.weight.dtype)
        for blk in self.encoder:
            x = blk(x, kpm if kpm.any() else None)
        return x, kpm

    def decode(self, tgt, memory, mem_kpm):
        y = self.tgt_emb(tgt) + self.pe[:tgt.shape[1]].to(self.tgt_emb.emb.weight.dtype)
        for blk in self.decoder:
            y = blk(y, memory, mem_kpm if mem_kpm.any() else None)
        return self.generator(y)

    def forward(self, src_input_ids, tgt_input_ids):
        memory, kpm = self.encode(src_input_ids)
        return self.decode(tgt_input_ids, memory, kpm)

    @torch.no_grad()
    def translate(self, src, bos_id: int, eos_id: int, max_len: int = 64):
        memory, kpm = self.encode(src)
        out = torch.full((src.shape[0], 1), bos_id, dtype=torch.long, device=src.device)
        for _ in range(max_len - 1):
            nxt = self.decode(out, memory, kpm)[:, -1].argmax(-1, keepdim=True)
            out = torch.cat([out, nxt], 1)
            if (nxt == eos_id).all():
                break
        return out


class DecoderOnlyTransformer(nn.Module):
    """cell 24 ``DecoderOnlyTransformer(vocab_size, d_model, num_heads, d_ff, num_layers=6)``."""

    def __init__(self, vocab_size: int, d_model: int = 64, num_heads: int = 4, d_ff: int = 256, num_layers: int = 6,
                 max_len: int = 5000, dropout: float = 0.0):
        super().__init__()
        self.emb = ScaledEmbedding(vocab_size, d_model)
        self.register_buffer("pe", sinusoidal_pe(max_len, d_model), persistent=False)
        self.blocks = nn.ModuleList([DecoderBlock(d_model, num_heads, d_ff, dropout, cross=False)
                                     for _ in range(num_layers)])
        self.lm_head = nn.Linear(d_model, vocab_size)

    def forward(self, input_ids):
        x = self.emb(input_ids) + self.pe[:input_ids.shape[1]].to(self.emb.emb.weight.dtype)
        for blk in self.blocks:
            x = blk(x)
        return self.lm_head(x)


# ------------------------------------------------------------------------------------ MiniBert
class _BertLayer(nn.Module):
    """cell 34 ``BertEncoderLayer``: pre-LN ``x + drop(attn(norm1(x), mask))``, ``x + drop(ffn(norm2(x)))``."""

    def __init__(self, hidden, heads, ffn, dropout):
        super().__init__()
        self.attn = MultiheadAttention(hidden, heads, dropout, batch_first=True)
        self.norm1, self.norm2 = LayerNorm(hidden), LayerNorm(hidden)
        self.ffn = _FF(hidden, ffn, dropout, act="gelu")
        self.drop = nn.Dropout(dropout)

    def forward(self, x, kpm=None):
        x = x + self.drop(self.attn(self.norm1(x), key_padding_mask=kpm)[0])
        return x + self.drop(self.ffn(self.norm2(x)))


class MiniBert(nn.Module):
    """cell 34 ``MiniBert(vocab_size, hidden_size=128, num_heads=4, num_layers=2, ffn_size=256,
    max_len=256, num_classes=2, dropout=0.1)``; ``mask`` is the tokenizer's attention_mask (1 = token)."""

    def __init__(self, vocab_size: int, hidden_size: int = 128, num_heads: int = 4, num_layers: int = 2,
                 ffn_size: int = 256, max_len: int = 256, num_classes: int = 2, dropout: float = 0.1):
        super().__init__()
        self.token_emb = Embedding(vocab_size, hidden_size)
        self.pos_emb = Embedding(max_len, hidden_size)
        self.dropout = nn.Dropout(dropout)
        self.layers = nn.ModuleList([_BertLayer(hidden_size, num_heads, ffn_size, dropout) for _ in range(num_layers)])
        self.norm = LayerNorm(hidden_size)
        self.classifier = nn.Linear(hidden_size, num_classes)

    def forward(self, x, mask=None):
        pos = torch.arange(x.shape[1], device=x.device)[None]
        h = self.dropout(self.token_emb(x) + self.pos_emb(pos))
        kpm = None if mask is None else (mask == 0)
        if kpm is not None and not kpm.any():
            kpm = None
        for layer in self.layers:
            h = layer(h, kpm)
        return self.classifier(self.norm(h)[:, 0])


# ------------------------------------------------------------------------------------ GPT (cells 39/41)
@dataclasses.dataclass
class NotebookGPTConfig:
    vocab_size: int = 50257       # GPT-2 tokenizer (cell 39); 21128 = bert-base-chinese (cell 41)
    n_embd: int = 256
    n_head: int = 8
    n_layer: int = 6
    max_seq_len: int = 128
    dropout: float = 0.1


class _GPTBlock(nn.Module):
    def __init__(self, c: NotebookGPTConfig):
        super().__init__()
        self.ln1, self.ln2 = LayerNorm(c.n_embd), LayerNorm(c.n_embd)
        self.attn = MultiheadAttention(c.n_embd, c.n_head, c.dropout, batch_first=True)
        self.mlp = _FF(c.n_embd, 4 * c.n_embd, c.dropout, act="gelu")
        self.drop = nn.Dropout(c.dropout)

    def forward(self, x):
        x = x + self.drop(self.attn(self.ln1(x), is_causal=True)[0])
        return x + self.drop(self.mlp(self.ln2(x)))


class NotebookGPT(nn.Module):
    """cells 39 / 41 ``MiniGPT(config)``: token + learned position embeddings, pre-LN blocks under a
    causal mask, final LayerNorm, LM head; ``generate`` samples with ``torch.multinomial``."""

    def __init__(self, config: NotebookGPTConfig):
        super().__init__()
        self.config = c = config
        self.tok_emb = Embedding(c.vocab_size, c.n_embd)
        self.pos_emb = Embedding(c.max_seq_len, c.n_embd)
        self.drop = nn.Dropout(c.dropout)
        self.blocks = nn.ModuleList([_GPTBlock(c) for _ in range(c.n_layer)])
        self.ln_f = LayerNorm(c.n_embd)
        self.head = nn.Linear(c.n_embd, c.vocab_size, bias=False)

    def forward(self, idx, targets=None):
        T = idx.shape[1]
        x = self.drop(self.tok_emb(idx) + self.pos_emb(torch.arange(T, device=idx.device))[None])
        for b in self.blocks:
            x = b(x)
        logits = self.head(self.ln_f(x))
        loss = None
        if targets is not None:
            loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), targets.reshape(-1), ignore_index=-100)
        return logits, loss

    @torch.no_grad()
    def generate(self, idx, max_new_tokens: int, temperature: float = 1.0, generator=None):
        for _ in range(max_new_tokens):
            logits, _ = self(idx[:, -self.config.max_seq_len:])
            probs = torch.softmax(logits[:, -1].float() / max(temperature, 1e-6), -1)
            idx = torch.cat([idx, torch.multinomial(probs, 1, generator=generator)], 1)
        return idx
