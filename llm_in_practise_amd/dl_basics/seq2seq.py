"""GRU Seq2Seq with Bahdanau (additive) attention (``DL_Basics/CNN_and_RNN.ipynb``: "Seq2Seq示例 —
简单的seq2seq模型 / 机器翻译模型示例 / SRE告警处理建议 / 日志分析与异常检测"), plus the variable-length
batching the notebooks build with ``DataLoader(collate_fn=…)`` and ``pack_padded_sequence``.

The notebooks train word-level toy pairs (English→French, alert text→remediation, log line→label);
:func:`train_seq2seq` takes any list of ``(source, target)`` strings, builds a character or
whitespace vocabulary, and trains with teacher forcing; :meth:`Seq2Seq.greedy_decode` generates.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence, pad_sequence

PAD, SOS, EOS, UNK = 0, 1, 2, 3


class Vocab:
    def __init__(self, texts: list[str], level: str = "char"):
        self.level = level
        toks = sorted({t for s in texts for t in self.split(s)})
        self.itos = ["<pad>", "<sos>", "<eos>", "<unk>"] + toks
        self.stoi = {t: i for i, t in enumerate(self.itos)}

    def split(self, s: str) -> list[str]:
        return list(s) if self.level == "char" else s.split()

    def encode(self, s: str) -> list[int]:
        return [self.stoi.get(t, UNK) for t in self.split(s)] + [EOS]

    def decode(self, ids: list[int]) -> str:
        out = []
        for i in ids:
            if i == EOS:
                break
            if i > UNK:
                out.append(self.itos[i])
        return ("" if self.level == "char" else " ").join(out)

    def __len__(self) -> int:
        return len(self.itos)


def pad_collate(batch: list[tuple[list[int], list[int]]]):
    """Collate ``(src_ids, tgt_ids)`` pairs into padded ``(B, S)`` / ``(B, T)`` tensors + source lengths."""
    src = [torch.tensor(s) for s, _ in batch]
    tgt = [torch.tensor(t) for _, t in batch]
    lens = torch.tensor([len(s) for s in src])
    return pad_sequence(src, batch_first=True, padding_value=PAD), lens, pad_sequence(tgt, batch_first=True,
                                                                                       padding_value=PAD)


class Encoder(nn.Module):
    def __init__(self, vocab: int, emb: int, hidden: int):
        super().__init__()
        self.emb = nn.Embedding(vocab, emb, padding_idx=PAD)
        self.rnn = nn.GRU(emb, hidden, batch_first=True, bidirectional=True)
        self.bridge = nn.Linear(2 * hidden, hidden)

    def forward(self, src, lens):
        packed = pack_padded_sequence(self.emb(src), lens.cpu(), batch_first=True, enforce_sorted=False)
        out, h = self.rnn(packed)
        out, _ = pad_packed_sequence(out, batch_first=True, total_length=src.shape[1])
        return out, torch.tanh(self.bridge(torch.cat([h[0], h[1]], dim=-1)))       # (B,S,2H), (B,H)


class BahdanauAttention(nn.Module):
    """score(s, h_j) = vᵀ tanh(W_s s + W_h h_j); masked softmax over source positions."""

    def __init__(self, dec_hidden: int, enc_dim: int, attn: int):
        super().__init__()
        self.w_s = nn.Linear(dec_hidden, attn, bias=False)
        self.w_h = nn.Linear(enc_dim, attn)
        self.v = nn.Linear(attn, 1, bias=False)

    def forward(self, s, enc_proj, enc_out, mask):
        e = self.v(torch.tanh(self.w_s(s)[:, None, :] + enc_proj)).squeeze(-1)     # (B,S)
        a = torch.softmax(e.masked_fill(~mask, float("-inf")), dim=-1)
        return torch.bmm(a[:, None, :], enc_out).squeeze(1), a


class Decoder(nn.Module):
    def __init__(self, vocab: int, emb: int, hidden: int, enc_dim: int):
        super().__init__()
        self.emb = nn.Embedding(vocab, emb, padding_idx=PAD)
        self.attn = BahdanauAttention(hidden, enc_dim, hidden)
        self.cell = nn.GRUCell(emb + enc_dim, hidden)
        self.out = nn.Linear(hidden + enc_dim + emb, vocab)

    def step(self, tok, h, enc_proj, enc_out, mask):
        e = self.emb(tok)
        ctx, a = self.attn(h, enc_proj, enc_out, mask)
        h = self.cell(torch.cat([e, ctx], -1), h)
        return self.out(torch.cat([h, ctx, e], -1)), h, a


class Seq2Seq(nn.Module):
    def __init__(self, src_vocab: int, tgt_vocab: int, emb: int = 32, hidden: int = 64):
        super().__init__()
        self.encoder = Encoder(src_vocab, emb, hidden)
        self.decoder = Decoder(tgt_vocab, emb, hidden, 2 * hidden)

    def forward(self, src, lens, tgt, teacher_forcing: float = 1.0):
        """Logits ``(B, T, V)`` for targets ``tgt`` (each row ends in EOS, PAD after)."""
        enc_out, h = self.encoder(src, lens)
        enc_proj = self.decoder.attn.w_h(enc_out)
        mask = src != PAD
        tok = torch.full((src.shape[0],), SOS, dtype=torch.long, device=src.device)
        logits = []
        for t in range(tgt.shape[1]):
            lo, h, _ = self.decoder.step(tok, h, enc_proj, enc_out, mask)
            logits.append(lo)
            use_tf = teacher_forcing >= 1.0 or torch.rand(()) < teacher_forcing
            tok = tgt[:, t] if use_tf else lo.argmax(-1)
        return torch.stack(logits, 1)

    @torch.no_grad()
    def greedy_decode(self, src, lens, max_len: int = 32):
        enc_out, h = self.encoder(src, lens)
        enc_proj = self.decoder.attn.w_h(enc_out)
        mask = src != PAD
        tok = torch.full((src.shape[0],), SOS, dtype=torch.long, device=src.device)
        out, attn = [], []
        for _ in range(max_len):
            lo, h, a = self.decoder.step(tok, h, enc_proj, enc_out, mask)
            tok = lo.argmax(-1)
            out.append(tok)
            attn.append(a)
        return torch.stack(out, 1), torch.stack(attn, 1)


def train_seq2seq(pairs: list[tuple[str, str]], *, level: str = "char", epochs: int = 30, batch_size: int = 32,
                  lr: float = 3e-3, emb: int = 32, hidden: int = 64, seed: int = 0, device: str = "cpu"):
    """Teacher-forced training with Adam + grad clipping 1.0; returns ``(model, src_vocab, tgt_vocab, losses)``."""
    torch.manual_seed(seed)
    sv, tv = Vocab([s for s, _ in pairs], level), Vocab([t for _, t in pairs], level)
    data = [(sv.encode(s), tv.encode(t)) for s, t in pairs]
    model = Seq2Seq(len(sv), len(tv), emb, hidden).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    loss_fn = nn.CrossEntropyLoss(ignore_index=PAD)
    loader = torch.utils.data.DataLoader(data, batch_size=batch_size, shuffle=True, collate_fn=pad_collate,
                                         generator=torch.Generator().manual_seed(seed))
    losses = []
    model.train()
    for _ in range(epochs):
        tot, n = 0.0, 0
        for src, lens, tgt in loader:
            src, lens, tgt = src.to(device), lens.to(device), tgt.to(device)
            logits = model(src, lens, tgt)
            loss = loss_fn(logits.reshape(-1, logits.shape[-1]), tgt.reshape(-1))
            opt.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            tot, n = tot + loss.item() * src.shape[0], n + src.shape[0]
        losses.append(tot / n)
    model.eval()
    return model, sv, tv, losses


def translate(model: Seq2Seq, sv: Vocab, tv: Vocab, texts: list[str], max_len: int = 32) -> list[str]:
    dev = next(model.parameters()).device
    src, lens, _ = pad_collate([(sv.encode(t), [EOS]) for t in texts])
    ids, _ = model.greedy_decode(src.to(dev), lens.to(dev), max_len)
    return [tv.decode(r.tolist()) for r in ids]
