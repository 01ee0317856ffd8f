"""Generation-time ops (SURVEY.md K16 sampling, K17 KV-cache decode attention).

GPU: ``csrc/kernels/decode.hip`` (split-K flash-decoding over the contiguous cache; fused
penalty/temperature/top-k/top-p/multinomial sampler).  CPU: the PyTorch references below, which
also define the semantics the kernels are tested against:

* repetition penalty — HF ``RepetitionPenaltyLogitsProcessor``: for every distinct token already
  in the sequence, ``s < 0 ? s * p : s / p`` (``GPTQModel/inference_qwen3_4b_gptq.py:16`` uses 1.1);
* temperature → top-k → top-p (HF warper order; top-p keeps the smallest top set whose mass is
  ``>= top_p``, at least one token), then a multinomial draw (``Fine-Tuning/inferences.py:51-58``);
* ``temperature <= 0`` or ``do_sample=False`` → greedy argmax (``llm-demo/minigpt/generate.py:25``).
"""
from __future__ import annotations

import math

import torch

from ._native import native, use_native


def decode_attention_reference(q, kc, vc, lens, hq, hkv, d, scale=None):
    """q [B, hq*d]; kc/vc [B, Smax, hkv*d]; lens [B] valid keys.  Returns [B, hq*d]."""
    B, Smax = kc.shape[0], kc.shape[1]
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    qf = q.float().view(B, hkv, hq // hkv, d)
    kf = kc.float().view(B, Smax, hkv, d)
    vf = vc.float().view(B, Smax, hkv, d)
    s = torch.einsum("bhgd,bshd->bhgs", qf, kf) * scale
    mask = torch.arange(Smax, device=q.device)[None, :] < lens.to(q.device)[:, None].long()
    s = s.masked_fill(~mask[:, None, None, :], float("-inf"))
    p = torch.nan_to_num(torch.softmax(s, -1), nan=0.0)
    o = torch.einsum("bhgs,bshd->bhgd", p, vf)
    return o.reshape(B, hq * d).to(q.dtype)


def decode_attention(q, kc, vc, lens, hq, hkv, d, max_len=None, scale=None):
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    G = hq // hkv if hkv else 0
    if (use_native(q) and q.dtype == torch.bfloat16 and d in (64, 128) and G in (1, 2, 4, 5, 8)
            and kc.is_contiguous() and vc.is_contiguous()):
        return native().decode_attention(q.contiguous(), kc, vc, lens.to(torch.int32).contiguous(), hq, hkv, d,
                                         int(max_len or kc.shape[1]), float(scale))
    return decode_attention_reference(q, kc, vc, lens, hq, hkv, d, scale)


def decode_attention_append(q, k, v, kc, vc, pos, hq, hkv, d, max_len=None, scale=None):
    """One decode step of every row: write ``k``/``v`` [B, hkv*d] into the caches at ``pos``
    [B] (int64) and attend ``q`` [B, hq*d] over the ``pos + 1`` keys.  On gfx950 one MFMA
    split-K kernel does both (``decode_attn_mfma_k``): the new rows are consumed from ``k``/``v``
    directly and stored by the split that holds the last key."""
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    G = hq // hkv if hkv else 0
    if (use_native(q) and q.dtype == torch.bfloat16 and d in (64, 128) and hq % hkv == 0 and 1 <= G <= 16
            and kc.is_contiguous() and vc.is_contiguous() and pos.dtype == torch.long
            and all(t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 for t in (q, k, v))):
        return native().decode_attention_append(q, k, v, kc, vc, pos.contiguous(), hq, hkv, d,
                                                int(max_len or kc.shape[1]), float(scale))
    rows = torch.arange(q.shape[0], device=q.device)
    kc[rows, pos] = k
    vc[rows, pos] = v
    return decode_attention(q, kc, vc, pos + 1, hq, hkv, d, max_len, scale)


def apply_repetition_penalty(logits: torch.Tensor, history: torch.Tensor | None, penalty: float) -> torch.Tensor:
    if history is None or penalty == 1.0:
        return logits
    h = history.long().clamp(min=0)
    hit = torch.zeros(logits.shape, dtype=torch.int32, device=logits.device)
    hit.scatter_add_(1, h, (history >= 0).to(torch.int32))     # pads (−1) contribute nothing
    pen = torch.where(logits < 0, logits * penalty, logits / penalty)
    return torch.where(hit > 0, pen, logits)


def sample_reference(logits, history=None, temperature=1.0, top_k=0, top_p=1.0, penalty=1.0, generator=None):
    x = apply_repetition_penalty(logits.float(), history, penalty)
    if not temperature or temperature <= 0:
        return torch.argmax(x, -1)
    x = x / temperature
    V = x.shape[-1]
    if top_k and 0 < top_k < V:
        kth = torch.topk(x, top_k, dim=-1).values[:, -1:]
        x = x.masked_fill(x < kth, float("-inf"))
    if top_p < 1.0:
        sx, si = torch.sort(x, dim=-1, descending=False)
        cum = torch.softmax(sx, -1).cumsum(-1)
        remove = cum <= (1 - top_p)
        remove[:, -1] = False
        x = x.scatter(1, si, sx.masked_fill(remove, float("-inf")))
    p = torch.softmax(x, -1)
    return torch.multinomial(p, 1, generator=generator).squeeze(-1)


_KEY = [0x5EED]


def sample(logits, history=None, temperature=1.0, top_k=0, top_p=1.0, penalty=1.0, key=None, generator=None):
    """One token per row.  ``history`` [B, L] int (−1 = padding) for the repetition penalty."""
    if use_native(logits) and logits.dtype in (torch.float32, torch.bfloat16):
        if key is None:
            _KEY[0] = (_KEY[0] * 6364136223846793005 + 1442695040888963407) & 0x7FFFFFFFFFFFFFFF
            key = _KEY[0]
        h = history.to(torch.int32).contiguous() if history is not None else None
        return native().sample(logits.contiguous(), h, float(temperature or 0.0), int(top_k or 0), float(top_p),
                               float(penalty), int(key))
    return sample_reference(logits, history, temperature, top_k, top_p, penalty, generator)


def seed_sampler(seed: int):
    _KEY[0] = (int(seed) * 0x9E3779B97F4A7C15 + 1) & 0x7FFFFFFFFFFFFFFF
