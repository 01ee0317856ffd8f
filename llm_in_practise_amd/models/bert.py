"""BERT encoder + sequence classification head (``HF_Basics/trainer_demo.py:61-119``,
BERT-base IMDb sentiment with ``Trainer``; B7 MiniBERT cells).

Parameter names follow the HF checkpoint layout (``bert.embeddings.word_embeddings.weight``,
``bert.encoder.layer.{i}.attention.self.query.weight``, …, ``classifier.weight``) so a local
``bert-base-uncased`` directory loads with :meth:`BertForSequenceClassification.from_pretrained`.
Compute runs on the framework's ops: fused LayerNorm / GELU kernels and the attention op with a
key-padding mask (post-LN encoder, erf GELU, pooler = tanh(dense(CLS))).
"""
from __future__ import annotations

import dataclasses
import json
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activation import gelu
from ..ops.attention import sdpa_bshd
from ..ops.norm import LayerNorm
from ..ops.embedding import Embedding


@dataclasses.dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    num_labels: int = 2
    pad_token_id: int = 0

    @classmethod
    def from_dict(cls, d):
        f = {x.name for x in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in f}
        if "id2label" in d and "num_labels" not in d:
            kw["num_labels"] = len(d["id2label"])
        return cls(**kw)


class _Embeddings(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.word_embeddings = Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.position_embeddings = Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)

    def forward(self, ids, token_type_ids=None):
        S = ids.shape[1]
        pos = torch.arange(S, device=ids.device)[None]
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(ids)
        x = self.word_embeddings(ids) + self.position_embeddings(pos) + self.token_type_embeddings(tt)
        return self.dropout(self.LayerNorm(x))


class _SelfAttn(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.query = nn.Linear(c.hidden_size, c.hidden_size)
        self.key = nn.Linear(c.hidden_size, c.hidden_size)
        self.value = nn.Linear(c.hidden_size, c.hidden_size)
        self.h, self.p = c.num_attention_heads, c.attention_probs_dropout_prob


class _SelfOut(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)
        self.LayerNorm = LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class _Attention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.self = _SelfAttn(c)
        self.output = _SelfOut(c)

    def forward(self, x, kpm):
        B, S, H = x.shape
        a = self.self
        d = H // a.h
        q = a.query(x).view(B, S, a.h, d)
        k = a.key(x).view(B, S, a.h, d)
        v = a.value(x).view(B, S, a.h, d)
        o = sdpa_bshd(q, k, v, causal=False, dropout_p=a.p if self.training else 0.0, key_padding_mask=kpm)
        o = self.output.dropout(self.output.dense(o.reshape(B, S, H)))
        return self.output.LayerNorm(o + x)


class _Intermediate(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.intermediate_size)


class _Output(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.intermediate_size, c.hidden_size)
        self.LayerNorm = LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class _Layer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.attention = _Attention(c)
        self.intermediate = _Intermediate(c)
        self.output = _Output(c)

    def forward(self, x, kpm):
        x = self.attention(x, kpm)
        h = gelu(self.intermediate.dense(x))
        return self.output.LayerNorm(self.output.dropout(self.output.dense(h)) + x)


class _Encoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layer = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


class _Pooler(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)

    def forward(self, x):
        return torch.tanh(self.dense(x[:, 0]))


class BertModel(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)
        self.pooler = _Pooler(c)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None):
        kpm = attention_mask.bool() if attention_mask is not None else None
        x = self.embeddings(input_ids, token_type_ids)
        for layer in self.encoder.layer:
            x = layer(x, kpm)
        return x, self.pooler(x)


@dataclasses.dataclass
class SequenceClassifierOutput:
    loss: torch.Tensor | None
    logits: torch.Tensor


class BertForSequenceClassification(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.config = c
        self.num_labels = c.num_labels
        self.bert = BertModel(c)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)
        self.classifier = nn.Linear(c.hidden_size, c.num_labels)
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=0.02)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None, labels=None, **_):
        _, pooled = self.bert(input_ids, attention_mask, token_type_ids)
        logits = self.classifier(self.dropout(pooled))
        loss = F.cross_entropy(logits.float(), labels) if labels is not None else None
        return SequenceClassifierOutput(loss, logits)

    @classmethod
    def from_pretrained(cls, path: str, num_labels: int = 2, device=None) -> "BertForSequenceClassification":
        """Local HF directory (``config.json`` + ``model.safetensors`` / ``pytorch_model.bin`` loaded
        with ``weights_only=True``); the classifier head is freshly initialised when absent."""
        with open(os.path.join(path, "config.json")) as f:
            d = json.load(f)
        d["num_labels"] = num_labels
        m = cls(BertConfig.from_dict(d))
        sd = {}
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        elif os.path.exists(os.path.join(path, "pytorch_model.bin")):
            sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
        sd = {k.replace(".gamma", ".weight").replace(".beta", ".bias"): v for k, v in sd.items()}
        own = m.state_dict()
        with torch.no_grad():
            for k, v in sd.items():
                if k in own and own[k].shape == v.shape:
                    own[k].copy_(v)
        return m.to(device or "cpu")


def accuracy_metric(eval_pred) -> dict:
    """``compute_metrics`` of the reference demo: accuracy of argmax predictions."""
    preds, labels = eval_pred
    preds = torch.as_tensor(preds).argmax(-1)
    return {"accuracy": float((preds == torch.as_tensor(labels)).float().mean())}
