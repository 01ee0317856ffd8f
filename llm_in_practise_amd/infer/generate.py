"""Autoregressive generation (reference call sites:
``Fine-Tuning/inferences.py:51-58`` (top-p 0.9, T 0.7), ``GPTQModel/inference_qwen3_4b_gptq.py:14-16``
(repetition penalty 1.1), ``llm-demo/minigpt/generate.py:14-29`` (greedy, sliding window),
``llm-demo/minigpt2/test_model.py:35-58`` (T 0.8 multinomial)).

Two paths:

* :func:`generate` — KV-cache decoding for the Qwen3 family (and anything exposing
  ``.model(input_ids, position_ids, cache, kv_lens)`` + ``.lm_head``).  Prompts are right-padded;
  prefill runs the fused flash-attention kernel with per-row key lengths, then every decode step
  appends one token per row at its own position (``KVCache.write_rows``) and runs the split-K
  decode-attention kernel; logits of the last position go through the fused sampler kernel.
  A decode step has no host synchronisation except the (optional) early-stop check, which is
  done every ``sync_every`` tokens.
* :func:`generate_simple` — the teaching models (MiniGPT, MiniGPT2, GPTLike, DeepSeekLike):
  no cache, the context is re-run over a sliding window exactly like the reference scripts.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Iterable

import torch

from ..models.common import KVCache
from ..ops.decode import sample


@dataclasses.dataclass
class GenerationConfig:
    max_new_tokens: int = 256
    do_sample: bool = False
    temperature: float = 1.0
    top_k: int = 0
    top_p: float = 1.0
    repetition_penalty: float = 1.0
    eos_token_id: int | list[int] | None = None
    pad_token_id: int | None = None
    seed: int | None = None
    sync_every: int = 8          # host check for "all rows finished" every N tokens

    @classmethod
    def from_kwargs(cls, base: "GenerationConfig | None" = None, **kw) -> "GenerationConfig":
        d = dataclasses.asdict(base) if base is not None else {}
        names = {f.name for f in dataclasses.fields(cls)}
        d.update({k: v for k, v in kw.items() if k in names and v is not None})
        return cls(**d)


def _unwrap_causal_lm(model):
    m = model
    for _ in range(4):
        if hasattr(m, "lm_head") and hasattr(m, "model"):
            return m
        m = getattr(m, "model", None) or getattr(m, "module", None)
        if m is None:
            break
    raise TypeError("generate() needs a causal LM with .model and .lm_head (e.g. Qwen3ForCausalLM)")


def _eos_set(eos) -> list[int]:
    if eos is None:
        return []
    return [int(eos)] if isinstance(eos, int) else [int(e) for e in eos]


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, attention_mask: torch.Tensor | None = None,
             generation_config: GenerationConfig | None = None, streamer=None, **kw) -> torch.Tensor:
    """Returns ``[B, S_max + new]``: row b = its prompt (right-padded region skipped) followed by
    its generated tokens, padded with ``pad_token_id`` after it finishes."""
    cfg = GenerationConfig.from_kwargs(generation_config, **kw)
    lm = _unwrap_causal_lm(model)
    was_training = lm.training
    lm.eval()
    dev = input_ids.device
    B, S = input_ids.shape
    if attention_mask is None:
        attention_mask = torch.ones_like(input_ids)
    lens = attention_mask.long().sum(1)
    mcfg = lm.config
    n_layers = mcfg.num_hidden_layers
    hkv, d = mcfg.num_key_value_heads, mcfg.head_dim
    cache = KVCache(n_layers, B, S + cfg.max_new_tokens, hkv, d, lm.lm_head.weight.dtype, dev)
    temperature = cfg.temperature if cfg.do_sample else 0.0
    if cfg.seed is not None:
        from ..ops.decode import seed_sampler
        seed_sampler(cfg.seed)
        torch.manual_seed(cfg.seed)
    eos = torch.tensor(_eos_set(cfg.eos_token_id) or [-1], device=dev)
    pad = cfg.pad_token_id if cfg.pad_token_id is not None else (int(eos[0]) if int(eos[0]) >= 0 else 0)

    # ---- prefill (right-padded prompts, per-row key lengths)
    kv_lens = lens.to(torch.int32)
    h = lm.model(input_ids, None, cache, kv_lens)                     # [B*S, H]
    last = h.view(B, S, -1)[torch.arange(B, device=dev), lens - 1]   # [B, H]
    logits = last @ lm.lm_head.weight.t()
    history = torch.full((B, S + cfg.max_new_tokens), -1, dtype=torch.int32, device=dev)
    history[:, :S] = torch.where(attention_mask.bool(), input_ids, torch.full_like(input_ids, -1)).to(torch.int32)
    cache.start_decode(lens)
    out = torch.full((B, cfg.max_new_tokens), pad, dtype=torch.long, device=dev)
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    n_gen = 0
    for t in range(cfg.max_new_tokens):
        tok = sample(logits, history if cfg.repetition_penalty != 1.0 else None, temperature, cfg.top_k, cfg.top_p,
                     cfg.repetition_penalty)
        tok = torch.where(done, torch.full_like(tok, pad), tok)
        out[:, t] = tok
        history[torch.arange(B, device=dev), (lens + t).clamp(max=history.shape[1] - 1)] = tok.to(torch.int32)
        done = done | torch.isin(tok, eos)
        n_gen = t + 1
        if streamer is not None:
            streamer.put(tok.detach().cpu())
        if (t + 1) % max(1, cfg.sync_every) == 0 or streamer is not None:
            if bool(done.all()):
                break
        if t + 1 == cfg.max_new_tokens:
            break
        hd = lm.model(tok[:, None], None, cache, None)                # decode step: [B, H]
        logits = hd @ lm.lm_head.weight.t()
    if streamer is not None:
        streamer.end()
    if was_training:
        lm.train()
    # assemble: prompt (valid part) + generated, right-padded
    res = torch.full((B, S + n_gen), pad, dtype=torch.long, device=dev)
    res[:, :S] = torch.where(attention_mask.bool(), input_ids, torch.full_like(input_ids, pad))
    idx = lens[:, None] + torch.arange(n_gen, device=dev)[None]
    res.scatter_(1, idx, out[:, :n_gen])
    return res


@torch.no_grad()
def generate_simple(model: torch.nn.Module, idx: torch.Tensor, max_new_tokens: int, block_size: int,
                    temperature: float = 0.0, top_k: int = 0, top_p: float = 1.0,
                    logits_fn: Callable[[torch.Tensor], torch.Tensor] | None = None,
                    eos_token_id: int | None = None, pad_left_to: int | None = None, pad_id: int = 0) -> torch.Tensor:
    """Sliding-window generation without a cache for the teaching models.

    ``temperature=0`` → greedy (``minigpt/generate.py:23-25``: ``input_seq[-16:]`` then argmax);
    ``pad_left_to`` left-pads the window with ``pad_id`` to a fixed length
    (``minigpt2/test_model.py:26-33``)."""
    model.eval()
    for _ in range(max_new_tokens):
        ctx = idx[:, -block_size:]
        if pad_left_to is not None and ctx.shape[1] < pad_left_to:
            ctx = torch.cat([torch.full((ctx.shape[0], pad_left_to - ctx.shape[1]), pad_id, dtype=ctx.dtype,
                                        device=ctx.device), ctx], 1)
        out = logits_fn(ctx) if logits_fn is not None else model(ctx)
        logits = out[0] if isinstance(out, tuple) else getattr(out, "logits", out)
        nxt = sample(logits[:, -1, :].float(), None, temperature, top_k, top_p, 1.0)
        idx = torch.cat([idx, nxt[:, None].to(idx.dtype)], 1)
        if eos_token_id is not None and bool((nxt == eos_token_id).all()):
            break
    return idx


class TextStreamer:
    """Prints decoded text as it is generated (HF ``TextStreamer`` analogue, batch 1)."""

    def __init__(self, tokenizer, skip_prompt: bool = True, **decode_kw):
        self.tok, self.kw = tokenizer, decode_kw
        self.ids: list[int] = []
        self.printed = 0

    def put(self, ids: torch.Tensor):
        self.ids.extend(int(i) for i in ids.reshape(-1)[:1])
        text = self.tok.decode(self.ids, **self.kw)
        print(text[self.printed:], end="", flush=True)
        self.printed = len(text)

    def end(self):
        print(flush=True)


class TextIteratorStreamer:
    """Queue-backed streamer: ``generate`` runs in a thread, the consumer iterates text deltas
    (HF ``TextIteratorStreamer`` analogue; used by the OpenAI server's SSE path and the web UI
    of ``Scripts/inference/06-*webui*.py:55-85``)."""

    def __init__(self, tokenizer, timeout: float | None = None, **decode_kw):
        import queue
        self.tok, self.kw, self.timeout = tokenizer, decode_kw, timeout
        self.q: "queue.Queue[str | None]" = queue.Queue()
        self.ids: list[int] = []
        self.sent = 0

    def put(self, ids: torch.Tensor):
        self.ids.extend(int(i) for i in ids.reshape(-1)[:1])
        text = self.tok.decode(self.ids, **self.kw)
        if len(text) > self.sent and not text.endswith("�"):
            self.q.put(text[self.sent:])
            self.sent = len(text)

    def end(self):
        text = self.tok.decode(self.ids, **self.kw)
        if len(text) > self.sent:
            self.q.put(text[self.sent:])
        self.q.put(None)

    def __iter__(self) -> Iterable[str]:
        while True:
            item = self.q.get(timeout=self.timeout)
            if item is None:
                return
            yield item
