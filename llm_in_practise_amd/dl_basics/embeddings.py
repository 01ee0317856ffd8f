"""Word-embedding setup (``DL_Basics/CNN_and_RNN.ipynb`` "词嵌入示例": randomly initialised
``nn.Embedding``, pre-trained GloVe vectors, BERT contextual embeddings).

:func:`load_glove` streams a GloVe text file (``word v1 … vD`` per line) keeping only the words of
the vocabulary; :func:`build_embedding` creates the ``nn.Embedding`` with GloVe rows where
available and N(0, σ²) rows elsewhere (σ matched to the loaded vectors), row ``pad_idx`` zero,
optionally frozen.  BERT embeddings: ``models/bert.py`` (``BertModel`` last hidden state).
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn


def load_glove(path: str, vocab: dict[str, int] | None = None, dim: int | None = None) -> dict[str, np.ndarray]:
    out: dict[str, np.ndarray] = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            if len(parts) < 2:
                continue
            word, vals = parts[0], parts[1:]
            if dim is not None and len(vals) != dim:
                continue                                   # malformed / header line
            if vocab is None or word in vocab:
                out[word] = np.asarray(vals, dtype=np.float32)
    return out


def build_embedding(vocab: dict[str, int], dim: int, glove_path: str | None = None, freeze: bool = False,
                    pad_idx: int | None = 0, seed: int = 0) -> tuple[nn.Embedding, int]:
    """Returns ``(embedding, n_pretrained_rows)``."""
    g = torch.Generator().manual_seed(seed)
    vecs = load_glove(glove_path, vocab, dim) if glove_path else {}
    std = float(np.std(np.stack(list(vecs.values())))) if vecs else 1.0
    w = torch.randn(max(vocab.values()) + 1, dim, generator=g) * std
    for word, v in vecs.items():
        w[vocab[word]] = torch.from_numpy(v)
    if pad_idx is not None:
        w[pad_idx] = 0.0
    emb = nn.Embedding.from_pretrained(w, freeze=freeze, padding_idx=pad_idx)
    return emb, len(vecs)
