"""Quantised-model quality checks.

``self_ppl`` reproduces the reference's "perplexity" (``LLM-Compressor/AWQ/eval_qwen3_4b_awq.py:31-66``):
greedy-generate up to 256 tokens per prompt, then exp(−mean of the top-1 log-probability of the
model's OWN generated tokens, skipping the first) — a self-confidence proxy, not dataset PPL; the
reference quotes ≈8.19 for unquantised Qwen3-4B and passes quantised models below 9.0
(``:76-80``).  ``dataset_ppl`` is the ordinary token-level perplexity on held-out ids.
"""
from __future__ import annotations

import math
from typing import Iterable

import torch

from ..infer.generate import generate

PASS_THRESHOLD = 9.0


@torch.no_grad()
def self_ppl(model, prompts: Iterable[torch.Tensor], max_new_tokens: int = 256, eos_token_id=None) -> float:
    lp_sum, n = 0.0, 0
    for p in prompts:
        p = p.view(1, -1)
        out = generate(model, p, max_new_tokens=max_new_tokens, eos_token_id=eos_token_id)
        S = p.shape[1]
        gen = out[:, S:]
        if gen.shape[1] < 2:
            continue
        logits = model(out).logits[:, S - 1:-1].float()          # position t predicts token t+1
        lp = torch.log_softmax(logits, -1).gather(-1, gen[..., None]).squeeze(-1)
        lp_sum += lp[:, 1:].sum().item()                          # skip the first generated token
        n += lp.shape[1] - 1
    return math.exp(-lp_sum / max(1, n))


@torch.no_grad()
def dataset_ppl(model, ids: torch.Tensor, block: int = 512) -> float:
    ids = ids.view(-1)
    nll, n = 0.0, 0
    for s in range(0, ids.numel() - 1, block):
        x = ids[s:s + block + 1][None]
        if x.shape[1] < 2:
            break
        out = model(x[:, :-1], labels=x[:, :-1])
        logits = model(x[:, :-1]).logits.float() if out.loss is None else None
        if out.loss is not None:
            k = x.shape[1] - 2
            nll += out.loss.item() * k
            n += k
        else:
            lp = torch.log_softmax(logits, -1).gather(-1, x[:, 1:, None]).squeeze(-1)
            nll -= lp.sum().item()
            n += lp.numel()
    return math.exp(nll / max(1, n))
