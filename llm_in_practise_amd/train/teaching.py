"""Training drivers for the Transformer_Basics notebook models (``models/teaching.py``).

* :func:`train_minibert_classifier` — cell 34: IMDb sentiment with MiniBert; ``collate_fn``
  pads each batch to its longest sequence (≤ ``max_len``), [CLS] first; CrossEntropy, Adam(lr 1e-3,
  weight_decay 1e-5), 2 epochs, batch 16; per-epoch train loss / accuracy and test accuracy.
  Offline: records come from a local JSONL/CSV (``text`` / ``label``) — the IMDb download of the
  notebook is not available here.
* :func:`train_notebook_gpt` — cells 39 / 41: token stream chunked into ``max_seq_len + 1``
  windows (x = w[:-1], y = w[1:]), AdamW(3e-4, wd 0.01), then ``generate`` a continuation
  (WikiText-2 with the GPT-2 vocabulary, or the Chinese CLUECorpusSmall with a char-level /
  bert-base-chinese vocabulary — any local corpus + tokenizer here).
* :func:`train_seq2seq` — cells 20-22's encoder-decoder on a synthetic transduction task
  (sequence reversal), teacher forcing, greedy ``translate``.
"""
from __future__ import annotations

import dataclasses
import math
import random

import torch
import torch.nn.functional as F

from ..models.teaching import MiniBert, NotebookGPT, NotebookGPTConfig, Seq2SeqTransformer
from ..utils.logging import get_logger


def _device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


# ------------------------------------------------------------------------------------ MiniBert
@dataclasses.dataclass
class MiniBertConfig:
    hidden_size: int = 128
    num_heads: int = 4
    num_layers: int = 2
    ffn_size: int = 256
    max_len: int = 256
    num_classes: int = 2
    dropout: float = 0.1
    lr: float = 1e-3
    weight_decay: float = 1e-5
    epochs: int = 2
    batch_size: int = 16
    seed: int = 0


def collate_classification(batch, tokenizer, max_len: int, cls_id: int, pad_id: int):
    """cell 34 ``collate_fn``: truncate, pad to the longest in the batch, attention mask, labels."""
    seqs = []
    for r in batch:
        ids = list(tokenizer.encode(r["text"], add_special_tokens=False))[:max_len - 1]
        seqs.append([cls_id] + ids)
    L = max(len(s) for s in seqs)
    ids = torch.full((len(seqs), L), pad_id, dtype=torch.long)
    mask = torch.zeros((len(seqs), L), dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, :len(s)] = torch.tensor(s)
        mask[i, :len(s)] = 1
    return ids, mask, torch.tensor([int(r["label"]) for r in batch], dtype=torch.long)


def train_minibert_classifier(train, test, tokenizer, cfg: MiniBertConfig = MiniBertConfig(), device=None,
                              cls_id: int | None = None, pad_id: int | None = None) -> dict:
    log = get_logger("lipa.minibert")
    device = device or _device()
    torch.manual_seed(cfg.seed)
    vocab = int(getattr(tokenizer, "vocab_size", 256))
    cls_id = cls_id if cls_id is not None else (getattr(tokenizer, "cls_token_id", None) or vocab)
    pad_id = pad_id if pad_id is not None else (getattr(tokenizer, "pad_token_id", None) or 0)
    model = MiniBert(max(vocab, cls_id + 1), cfg.hidden_size, cfg.num_heads, cfg.num_layers, cfg.ffn_size,
                     cfg.max_len, cfg.num_classes, cfg.dropout).to(device)
    if device.type == "cuda":
        model.to(torch.bfloat16)
    opt = torch.optim.Adam(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    rng = random.Random(cfg.seed)
    hist = {"train_loss": [], "train_acc": [], "test_acc": []}
    for ep in range(cfg.epochs):
        order = list(range(len(train)))
        rng.shuffle(order)
        model.train()
        tot_l = tot_a = n = 0
        for s in range(0, len(order), cfg.batch_size):
            ids, mask, y = collate_classification([train[i] for i in order[s:s + cfg.batch_size]], tokenizer,
                                                  cfg.max_len, cls_id, pad_id)
            ids, mask, y = ids.to(device), mask.to(device), y.to(device)
            logits = model(ids, mask).float()
            loss = F.cross_entropy(logits, y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            tot_l += loss.item() * len(y)
            tot_a += (logits.argmax(-1) == y).sum().item()
            n += len(y)
        hist["train_loss"].append(tot_l / max(1, n))
        hist["train_acc"].append(tot_a / max(1, n))
        hist["test_acc"].append(evaluate_classifier(model, test, tokenizer, cfg, device, cls_id, pad_id))
        log.info("epoch %d train loss %.4f acc %.4f test acc %.4f", ep + 1, hist["train_loss"][-1],
                 hist["train_acc"][-1], hist["test_acc"][-1])
    hist["model"] = model
    return hist


@torch.no_grad()
def evaluate_classifier(model, data, tokenizer, cfg, device, cls_id, pad_id) -> float:
    model.eval()
    correct = total = 0
    for s in range(0, len(data), cfg.batch_size):
        ids, mask, y = collate_classification(data[s:s + cfg.batch_size], tokenizer, cfg.max_len, cls_id, pad_id)
        pred = model(ids.to(device), mask.to(device)).argmax(-1).cpu()
        correct += (pred == y).sum().item()
        total += len(y)
    return correct / max(1, total)


# ------------------------------------------------------------------------------------ notebook GPT
def train_notebook_gpt(texts: list[str], tokenizer, cfg: NotebookGPTConfig | None = None, epochs: int = 1,
                       batch_size: int = 16, lr: float = 3e-4, weight_decay: float = 0.01, max_steps: int = -1,
                       prompt: str | None = None, gen_tokens: int = 32, device=None, seed: int = 0) -> dict:
    log = get_logger("lipa.nbgpt")
    device = device or _device()
    torch.manual_seed(seed)
    ids: list[int] = []
    eos = getattr(tokenizer, "eos_token_id", None)
    for t in texts:
        ids.extend(tokenizer.encode(t, add_special_tokens=False))
        if eos is not None:
            ids.append(eos)
    cfg = cfg or NotebookGPTConfig(vocab_size=int(getattr(tokenizer, "vocab_size", 256)))
    T = cfg.max_seq_len
    n = (len(ids) - 1) // T
    if n < 1:
        raise ValueError(f"corpus too small: {len(ids)} tokens for max_seq_len {T}")
    data = torch.tensor(ids[:n * T + 1], dtype=torch.long)
    windows = torch.stack([data[i * T:(i + 1) * T + 1] for i in range(n)])
    model = NotebookGPT(cfg).to(device)
    if device.type == "cuda":
        model.to(torch.bfloat16)
    opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)
    g = torch.Generator().manual_seed(seed)
    losses, step = [], 0
    for ep in range(epochs):
        perm = torch.randperm(n, generator=g)
        model.train()
        for s in range(0, n, batch_size):
            w = windows[perm[s:s + batch_size]].to(device)
            _, loss = model(w[:, :-1], w[:, 1:])
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            losses.append(loss.item())
            step += 1
            if max_steps > 0 and step >= max_steps:
                break
        log.info("epoch %d loss %.4f ppl %.2f", ep + 1, losses[-1], math.exp(min(20, losses[-1])))
        if max_steps > 0 and step >= max_steps:
            break
    out = {"losses": losses, "model": model, "steps": step}
    if prompt is not None:
        model.eval()
        p = torch.tensor([tokenizer.encode(prompt, add_special_tokens=False)], device=device)
        gen = model.generate(p, gen_tokens, generator=torch.Generator(device=device).manual_seed(seed))
        out["sample"] = tokenizer.decode(gen[0].tolist())
    return out


# ------------------------------------------------------------------------------------ seq2seq
def reversal_batch(n: int, length: int, vocab: int, rng: random.Random, pad=0, bos=1, eos=2):
    src, tgt = [], []
    for _ in range(n):
        L = rng.randint(2, length)
        s = [rng.randrange(3, vocab) for _ in range(L)]
        src.append(s + [eos] + [pad] * (length - L))
        t = [bos] + s[::-1] + [eos]
        tgt.append(t + [pad] * (length + 2 - len(t)))
    return torch.tensor(src), torch.tensor(tgt)


def train_seq2seq(steps: int = 300, vocab: int = 12, length: int = 6, d_model: int = 64, num_heads: int = 4,
                  d_ff: int = 128, num_layers: int = 2, lr: float = 1e-3, batch: int = 64, device=None, seed: int = 0):
    """Teacher-forced training of the encoder-decoder Transformer on sequence reversal; returns
    (model, loss curve, exact-match accuracy of greedy ``translate`` on fresh samples)."""
    device = device or _device()
    torch.manual_seed(seed)
    rng = random.Random(seed)
    m = Seq2SeqTransformer(vocab, vocab, d_model, num_heads, d_ff, num_layers, max_len=64).to(device)
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    losses = []
    for _ in range(steps):
        src, tgt = (t.to(device) for t in reversal_batch(batch, length, vocab, rng))
        logits = m(src, tgt[:, :-1])
        loss = F.cross_entropy(logits.reshape(-1, vocab).float(), tgt[:, 1:].reshape(-1), ignore_index=0)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    m.eval()
    src, tgt = (t.to(device) for t in reversal_batch(128, length, vocab, random.Random(seed + 1)))
    out = m.translate(src, 1, 2, max_len=length + 2)
    ok = 0
    for o, t in zip(out.tolist(), tgt.tolist()):
        want = t[:t.index(2) + 1]
        ok += o[:len(want)] == want
    return m, losses, ok / len(out)
