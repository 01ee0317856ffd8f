"""Pure-PyTorch fp32 reference implementations of every native op.

These are (1) the CPU execution path (tests, the minigpt plumbing config) and (2) the
numerics oracle the HIP kernels are tested against.  Each function is
the plain math — no fusion, no tricks.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, weight: torch.Tensor | None, eps: float = 1e-6) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    if weight is not None:
        y = y * weight.float()
    return y.to(x.dtype)


def layernorm(x, weight, bias, eps: float = 1e-5):
    return F.layer_norm(x.float(), (x.shape[-1],), None if weight is None else weight.float(),
                        None if bias is None else bias.float(), eps).to(x.dtype)


# ----------------------------------------------------------------------------- rope
def rope_cos_sin(positions: torch.Tensor, dim: int, theta: float = 10000.0,
                 scaling: dict | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """cos/sin tables ``[len(positions), dim//2]`` (fp32), optional YaRN scaling."""
    inv_freq, attn_factor = rope_inv_freq(dim, theta, scaling)
    ang = positions.float()[:, None] * inv_freq.to(positions.device)[None, :]
    return torch.cos(ang) * attn_factor, torch.sin(ang) * attn_factor


def rope_inv_freq(dim: int, theta: float, scaling: dict | None = None):
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    attn_factor = 1.0
    if scaling and scaling.get("rope_type", scaling.get("type")) == "yarn":
        # YaRN (NTK-by-parts) [ext]: blend interpolated / extrapolated frequencies
        factor = float(scaling["factor"])
        orig = float(scaling.get("original_max_position_embeddings", 32768))
        beta_fast, beta_slow = float(scaling.get("beta_fast", 32)), float(scaling.get("beta_slow", 1))

        def corr_dim(nrot):
            return (dim * math.log(orig / (nrot * 2 * math.pi))) / (2 * math.log(theta))
        low = max(math.floor(corr_dim(beta_fast)), 0)
        high = min(math.ceil(corr_dim(beta_slow)), dim - 1)
        if low == high:
            high += 0.001
        ramp = (torch.arange(dim // 2, dtype=torch.float64) - low) / (high - low)
        extrap_w = 1 - ramp.clamp(0, 1)
        inv = (inv / factor) * (1 - extrap_w) + inv * extrap_w
        attn_factor = scaling.get("attention_factor") or (0.1 * math.log(factor) + 1.0)
    elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
        inv = inv / float(scaling["factor"])
    return inv.float(), float(attn_factor)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, interleaved: bool = False) -> torch.Tensor:
    """x: [..., S, H, D] with cos/sin [S, D/2].  rotate-half (Qwen/Llama) or interleaved
    pairs (DeepSeekLike complex form, ``DeepSeekLike_wikitext2.py:122-163``)."""
    xf = x.float()
    c = cos[:, None, :]
    s = sin[:, None, :]
    if interleaved:
        x1, x2 = xf[..., 0::2], xf[..., 1::2]
        o1, o2 = x1 * c - x2 * s, x2 * c + x1 * s
        return torch.stack([o1, o2], -1).flatten(-2).to(x.dtype)
    h = xf.shape[-1] // 2
    x1, x2 = xf[..., :h], xf[..., h:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).to(x.dtype)


# ----------------------------------------------------------------------------- activations
def swiglu(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    return (F.silu(gate.float()) * up.float()).to(gate.dtype)


def gelu(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float()).to(x.dtype)


# ----------------------------------------------------------------------------- attention
def attention(q, k, v, causal: bool = True, key_padding_mask: torch.Tensor | None = None,
              scale: float | None = None, window: int | None = None, dropout_p: float = 0.0):
    """q [B,S,Hq,D], k/v [B,S,Hkv,D] (GQA by head broadcast).  ``key_padding_mask`` [B,S]
    True = keep.  Returns [B,S,Hq,D]."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    mask = torch.zeros(S, Sk, dtype=torch.bool, device=q.device)
    if causal:
        mask |= torch.ones(S, Sk, dtype=torch.bool, device=q.device).triu(Sk - S + 1)
    if window is not None:
        i = torch.arange(S, device=q.device)[:, None] + (Sk - S)
        j = torch.arange(Sk, device=q.device)[None, :]
        mask |= (i - j) > window
    s = s.masked_fill(mask, float("-inf"))
    if key_padding_mask is not None:
        s = s.masked_fill(~key_padding_mask[:, None, None, :].bool(), float("-inf"))
    p = torch.softmax(s, -1)
    p = torch.nan_to_num(p, nan=0.0)
    if dropout_p > 0:
        p = F.dropout(p, dropout_p)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


# ----------------------------------------------------------------------------- loss
def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100,
                  reduction: str = "mean") -> torch.Tensor:
    return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), labels.view(-1),
                           ignore_index=ignore_index, reduction=reduction)


# ----------------------------------------------------------------------------- linear / lora
def lora_linear(x, w, lora_a=None, lora_b=None, scaling: float = 1.0, bias=None):
    """y = x Wᵀ (+ b) + s·(x Aᵀ) Bᵀ in fp32."""
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if lora_a is not None:
        y = y + scaling * ((x.float() @ lora_a.float().t()) @ lora_b.float().t())
    return y.to(x.dtype)


# ----------------------------------------------------------------------------- optimizers
def adamw_step(p, g, m, v, step: int, lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float):
    """In-place decoupled-weight-decay AdamW on fp32 tensors (torch.optim.AdamW semantics)."""
    p.mul_(1 - lr * weight_decay)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v / bc2).sqrt().add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
