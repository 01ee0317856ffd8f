"""Data pipelines (SURVEY.md X17, E-track SFT pipeline, A/B/C datasets).

SFT (``Fine-Tuning/qwen3-*-qlora*.py``): self-cognition records → placeholder substitution →
3-turn messages → ChatML → tokenize (max_length 512) → labels.  The reference's label masking
is reproduced bit-for-bit by default (``label_mode="reference"``) and its effective objective
is documented: masking ``labels[:first <|im_start|>]`` masks nothing, and
``DataCollatorForLanguageModeling(mlm=False)`` rebuilds ``labels = input_ids`` with every pad
(= eos = ``<|im_end|>``) set to -100, so training is plain causal-LM loss over non-pad tokens
(SURVEY §2.1 "SFT-pipeline behaviour").  ``label_mode="assistant"`` is the corrected
objective (loss only on assistant tokens) and pairs with :class:`DataCollatorForSeq2Seq`.

Pretraining datasets: ``TokenBlockDataset`` (concatenate → [N, block] → x=block[:-1],
y=block[1:], ``ddp_gpt_wikitext2.py:56-81``), ``CharWindowDataset`` (minigpt, ``train.py:15-22``),
``ByteBlocksDataset`` (C4, UTF-8 bytes), ``SyntheticLMDataset`` (benchmarks).
Tokenizers: HF ``tokenizers`` / ``transformers`` from LOCAL files only, plus char / byte
tokenizers and BPE training (``GPTLike_wikitext2.py:49-62``, ``fixed_pe.py:52-80``).
"""
from __future__ import annotations

import json
import os
from typing import Iterable, Sequence

import torch
from torch.utils.data import Dataset

QWEN3_SYSTEM = "你是一个有帮助的智能助手，由马哥教育AI团队训练，名为马哥教育AI小助手，旨在提供准确且友好的回答。"
DEEPSEEK_R1_SYSTEM = "该助手为DeepSeek-R1，由深度求索公司创造。今天是2025年10月23日。"
DEFAULT_NAME, DEFAULT_AUTHOR = "马哥教育AI小助手", "马哥教育AI团队"


# ============================================================================ SFT records
def load_records(path: str) -> list[dict]:
    """jsonl / json list (self-cognition schema: query, response, tag)."""
    with open(path, encoding="utf-8") as f:
        txt = f.read().strip()
    if txt.startswith("["):
        return json.loads(txt)
    return [json.loads(line) for line in txt.splitlines() if line.strip()]


def synthetic_self_cognition(n: int = 108, seed: int = 0) -> list[dict]:
    """Offline stand-in with the modelscope/self-cognition schema (108 rows like the original)."""
    import random
    rnd = random.Random(seed)
    qs = ["你是？", "你是谁!", "你好", "介绍一下你自己", "who are you?", "What is your name?", "你叫什么名字",
          "你是由谁开发的？", "Are you ChatGPT?", "你能做什么"]
    rs = ["我是{{NAME}}，由{{AUTHOR}}训练的人工智能助手。", "您好！我是{{AUTHOR}}开发的人工智能语言模型，名为{{NAME}}。",
          "I am {{NAME}}, an AI assistant developed by {{AUTHOR}}.", "我是{{NAME}}，可以回答您的问题、提供信息。"]
    return [{"query": rnd.choice(qs), "response": rnd.choice(rs), "tag": "zh" if i % 2 == 0 else "en"}
            for i in range(n)]


def replace_placeholders(rec: dict, name: str = DEFAULT_NAME, author: str = DEFAULT_AUTHOR) -> dict:
    r = dict(rec)
    r["response"] = r["response"].replace("{{NAME}}", name).replace("{{AUTHOR}}", author)
    return r


def to_chat_messages(rec: dict, system: str = QWEN3_SYSTEM) -> list[dict]:
    return [{"role": "system", "content": system}, {"role": "user", "content": rec["query"]},
            {"role": "assistant", "content": rec["response"]}]


def render_chatml(messages: Sequence[dict], space_before_end: bool = False, add_generation_prompt: bool = False,
                  strip: bool = True) -> str:
    """``<|im_start|>{role}\\n{content}<|im_end|>\\n`` per turn.  ``space_before_end`` selects the
    ``"{content} <|im_end|>"`` variant used by E2/E3/E8 (``qwen3-8b-qlora-dist.py:47``,
    ``inferences.py:40-46``)."""
    sep = " " if space_before_end else ""
    s = "".join(f"<|im_start|>{m['role']}\n{m['content']}{sep}<|im_end|>\n" for m in messages)
    if add_generation_prompt:
        return s + "<|im_start|>assistant\n"
    return s.strip() if strip else s


class SFTDataset(Dataset):
    """Tokenised ChatML SFT examples (lists of ids; padding done here or by the collator)."""

    def __init__(self, records: Iterable[dict], tokenizer, max_length: int = 512, padding: str = "max_length",
                 label_mode: str = "reference", system: str = QWEN3_SYSTEM, space_before_end: bool = False,
                 name: str = DEFAULT_NAME, author: str = DEFAULT_AUTHOR):
        self.tok = tokenizer
        pad_id = _pad_id(tokenizer)
        self.examples = []
        texts = [render_chatml(to_chat_messages(replace_placeholders(r, name, author), system), space_before_end)
                 for r in records]
        enc = [tokenizer.encode(t, add_special_tokens=False)[:max_length] for t in texts]
        width = max_length if padding == "max_length" else max(len(e) for e in enc)
        im_start = _token_id(tokenizer, "<|im_start|>")
        im_end = _token_id(tokenizer, "<|im_end|>")
        for ids in enc:
            n = len(ids)
            ids = ids + [pad_id] * (width - n)
            attn = [1] * n + [0] * (width - n)
            labels = list(ids)
            if label_mode == "reference":
                # labels[:first <|im_start|>] = -100 → first occurrence is position 0 (system turn)
                if im_start in ids:
                    first = ids.index(im_start)
                    labels[:first] = [-100] * first
            elif label_mode == "assistant":
                labels = _assistant_only_labels(ids, n, tokenizer, im_start, im_end)
            self.examples.append({"input_ids": ids, "attention_mask": attn, "labels": labels})

    def __len__(self):
        return len(self.examples)

    def __getitem__(self, i):
        return self.examples[i]


def _assistant_only_labels(ids, n, tok, im_start, im_end):
    labels = [-100] * len(ids)
    asst = tok.encode("assistant", add_special_tokens=False)
    i = 0
    while i < n:
        if ids[i] == im_start and ids[i + 1:i + 1 + len(asst)] == asst:
            j = i + 1 + len(asst)
            while j < n and ids[j] != im_end:
                labels[j] = ids[j]
                j += 1
            if j < n:
                labels[j] = ids[j]          # learn to emit <|im_end|>
            i = j
        i += 1
    return labels


def _pad_id(tok) -> int:
    pid = getattr(tok, "pad_token_id", None)
    if pid is None:
        pid = getattr(tok, "eos_token_id", None)
    return 0 if pid is None else int(pid)


def _token_id(tok, s: str):
    try:
        ids = tok.encode(s, add_special_tokens=False)
        return ids[0] if ids else None
    except Exception:
        return None


class DataCollatorForLanguageModeling:
    """HF ``DataCollatorForLanguageModeling(mlm=False)`` semantics [ext]: pad, then
    ``labels = input_ids`` with pad ids → -100 (any provided labels are discarded)."""

    def __init__(self, tokenizer=None, mlm: bool = False, pad_to_multiple_of: int | None = None,
                 pad_token_id: int | None = None):
        assert not mlm, "masked-LM collation is not part of this stack"
        self.pad_id = pad_token_id if pad_token_id is not None else _pad_id(tokenizer)
        self.mult = pad_to_multiple_of

    def __call__(self, batch: list[dict]) -> dict:
        ids, attn = _pad([b["input_ids"] for b in batch], self.pad_id, self.mult), None
        if "attention_mask" in batch[0]:
            attn = _pad([b["attention_mask"] for b in batch], 0, self.mult)
        labels = ids.clone()
        labels[ids == self.pad_id] = -100
        out = {"input_ids": ids, "labels": labels}
        if attn is not None:
            out["attention_mask"] = attn
        return out


class DataCollatorWithPadding:
    """Pad ``input_ids`` / ``attention_mask`` / ``token_type_ids`` to the longest row of the batch
    (``HF_Basics/trainer_demo.py``: dynamic padding for classification); ``label(s)`` stacked."""

    def __init__(self, tokenizer=None, pad_to_multiple_of: int | None = None, pad_token_id: int | None = None):
        self.pad = pad_token_id if pad_token_id is not None else (_pad_id(tokenizer) if tokenizer is not None else 0)
        self.mult = pad_to_multiple_of

    def __call__(self, batch):
        out = {"input_ids": _pad([b["input_ids"] for b in batch], self.pad, self.mult)}
        n = out["input_ids"].shape[1]
        if "attention_mask" in batch[0]:
            out["attention_mask"] = _pad([b["attention_mask"] for b in batch], 0, self.mult)[:, :n]
        else:
            out["attention_mask"] = _pad([[1] * len(b["input_ids"]) for b in batch], 0, self.mult)[:, :n]
        if "token_type_ids" in batch[0]:
            out["token_type_ids"] = _pad([b["token_type_ids"] for b in batch], 0, self.mult)[:, :n]
        for key in ("labels", "label"):
            if key in batch[0]:
                out["labels"] = torch.tensor([int(b[key]) for b in batch])
        return out


class DataCollatorForSeq2Seq:
    """Pads and keeps the provided labels (pad → -100): the corrected-objective collator."""

    def __init__(self, tokenizer=None, pad_to_multiple_of: int | None = None, pad_token_id: int | None = None):
        self.pad_id = pad_token_id if pad_token_id is not None else _pad_id(tokenizer)
        self.mult = pad_to_multiple_of

    def __call__(self, batch):
        return {"input_ids": _pad([b["input_ids"] for b in batch], self.pad_id, self.mult),
                "attention_mask": _pad([b["attention_mask"] for b in batch], 0, self.mult),
                "labels": _pad([b["labels"] for b in batch], -100, self.mult)}


def _pad(seqs, value, mult=None) -> torch.Tensor:
    seqs = [list(s) if not torch.is_tensor(s) else s.tolist() for s in seqs]
    w = max(len(s) for s in seqs)
    if mult:
        w = (w + mult - 1) // mult * mult
    return torch.tensor([s + [value] * (w - len(s)) for s in seqs], dtype=torch.long)


# ============================================================================ LM datasets
class TokenBlockDataset(Dataset):
    """Concatenate ids, keep a multiple of ``block_size`` and return ``(block[:-1], block[1:])``."""

    def __init__(self, ids: Sequence[int] | torch.Tensor, block_size: int):
        t = torch.as_tensor(ids, dtype=torch.long).reshape(-1)
        n = t.numel() // block_size
        self.data = t[: n * block_size].view(n, block_size)

    def __len__(self):
        return self.data.shape[0]

    def __getitem__(self, i):
        blk = self.data[i]
        return blk[:-1], blk[1:]


class CharWindowDataset(Dataset):
    """minigpt: sliding windows of ``seq_len`` chars, augmented ``repeat`` times
    (``llm-demo/minigpt/train.py:15-22``)."""

    def __init__(self, text: str, char2idx: dict, seq_len: int = 16, repeat: int = 10):
        self.items = []
        for _ in range(repeat):
            for i in range(len(text) - seq_len):
                x = [char2idx[c] for c in text[i:i + seq_len]]
                y = [char2idx[c] for c in text[i + 1:i + seq_len + 1]]
                self.items.append((torch.tensor(x), torch.tensor(y)))

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


class ByteBlocksDataset(TokenBlockDataset):
    """UTF-8 bytes as tokens (vocab 256, ``temp/ddp_gpt_wikitext2.py:79-116``)."""

    def __init__(self, texts: Iterable[str], block_size: int):
        data = bytearray()
        for t in texts:
            data.extend(t.encode("utf-8"))
        super().__init__(torch.tensor(list(data), dtype=torch.long), block_size)


class SyntheticLMDataset(Dataset):
    """Random token ids at a fixed shape (benchmarks: BASELINE.json prescribes synthetic data)."""

    def __init__(self, vocab: int, seq_len: int, n: int, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.ids = torch.randint(0, vocab, (n, seq_len), generator=g)

    def __len__(self):
        return self.ids.shape[0]

    def __getitem__(self, i):
        x = self.ids[i].tolist()
        return {"input_ids": x, "attention_mask": [1] * len(x), "labels": x}


# ============================================================================ tokenizers
class CharTokenizer:
    def __init__(self, text: str | None = None, stoi: dict | None = None):
        chars = sorted(set(text)) if stoi is None else None
        self.stoi = stoi or {c: i for i, c in enumerate(chars)}
        self.itos = {i: c for c, i in self.stoi.items()}
        self.vocab_size = len(self.stoi)
        self.pad_token_id = self.eos_token_id = None

    def encode(self, s, add_special_tokens=False):
        return [self.stoi[c] for c in s]

    def decode(self, ids, skip_special_tokens=True):
        return "".join(self.itos[int(i)] for i in ids)


class ByteTokenizer:
    vocab_size = 256
    pad_token_id = 0
    eos_token_id = 0

    def encode(self, s, add_special_tokens=False):
        return list(s.encode("utf-8"))

    def decode(self, ids, skip_special_tokens=True):
        return bytes(int(i) for i in ids if 0 <= int(i) < 256).decode("utf-8", errors="replace")


def train_bpe_tokenizer(texts: Iterable[str], vocab_size: int = 3000, kind: str = "whitespace",
                        special_tokens=("[PAD]", "[UNK]", "[BOS]", "[EOS]"), save_path: str | None = None):
    """BPE training with HF ``tokenizers`` — ``kind="whitespace"`` (B1) or ``"bytelevel"`` (B2/C5)."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    if kind == "bytelevel":
        tok = Tokenizer(models.BPE(unk_token=None))
        tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
        tok.decoder = decoders.ByteLevel()
        tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=list(special_tokens),
                                 initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    else:
        tok = Tokenizer(models.BPE(unk_token="[UNK]"))
        tok.pre_tokenizer = pre_tokenizers.Whitespace()
        tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=list(special_tokens))
    tok.train_from_iterator(texts, tr)
    if save_path:
        os.makedirs(os.path.dirname(save_path) or ".", exist_ok=True)
        tok.save(save_path)
    return HFTokenizerWrapper(tok)


class HFTokenizerWrapper:
    """Minimal encode/decode surface over a ``tokenizers.Tokenizer``."""

    def __init__(self, tok):
        self.tok = tok
        self.vocab_size = tok.get_vocab_size()
        self.pad_token_id = tok.token_to_id("[PAD]")
        self.eos_token_id = tok.token_to_id("[EOS]")

    @classmethod
    def from_file(cls, path):
        from tokenizers import Tokenizer
        return cls(Tokenizer.from_file(path))

    def encode(self, s, add_special_tokens=False):
        return self.tok.encode(s).ids

    def decode(self, ids, skip_special_tokens=True):
        return self.tok.decode([int(i) for i in ids], skip_special_tokens=skip_special_tokens)


def load_tokenizer(path: str, pad_to_eos: bool = True):
    """HF tokenizer from a LOCAL directory (no hub access); pad defaults to eos like the reference.
    ``"bytes"`` gives the UTF-8 byte tokenizer (random-init demos and tests, vocab 256)."""
    if path == "bytes":
        return ByteTokenizer()
    from transformers import AutoTokenizer
    tok = AutoTokenizer.from_pretrained(path, local_files_only=True, trust_remote_code=False)
    if pad_to_eos and tok.pad_token is None:
        tok.pad_token = tok.eos_token
    return tok


def load_text_corpus(path: str, field: str = "text") -> list[str]:
    """Local text corpus: .txt (one doc per line), .jsonl/.json (``field``), .parquet."""
    if path.endswith(".parquet"):
        import pyarrow.parquet as pq
        return [t for t in pq.read_table(path).column(field).to_pylist() if t and t.strip()]
    if path.endswith((".jsonl", ".json")):
        return [r[field] for r in load_records(path) if r.get(field, "").strip()]
    with open(path, encoding="utf-8") as f:
        return [line for line in f.read().splitlines() if line.strip()]
