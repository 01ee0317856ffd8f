"""AWQ W4A16: ``AWQModifier(targets="Linear", scheme="W4A16", ignore=["lm_head"])``
(``LLM-Compressor/AWQ/quantize_qwen3_4b_awq.py:17-25``) — activation-aware per-input-channel
scaling, then asymmetric group-128 int4.

For each (smooth op → balance linears) mapping of a Qwen3 decoder layer
  input_layernorm → q/k/v,  v_proj → o_proj (only when shapes match: skipped under GQA),
  post_attention_layernorm → gate/up,  up_proj → down_proj,
the calibration inputs X of the balance linears give the channel magnitude ``x̄ = mean|X|``;
for α on a grid in [0, 1) the candidate scale ``s = x̄^α / w̄^(1−α)`` (normalised to unit
geometric range) is scored by ‖X·Wᵀ − X·(Q(W·s)/s)ᵀ‖²; the best s is folded into the weights
(W·s for the balance linears, ÷s into the smooth op), which leaves the fp model's function
unchanged while moving quantisation error away from salient channels.  Finally every decoder
linear is RTN-quantised (the AWQ scales having done the work).
"""
from __future__ import annotations

from typing import Iterable

import torch
import torch.nn as nn

from .calib import LayerWalker, get_module
from .gptq import replace_with_int4
from .int4 import Int4Weight, quant_params, quantize_rtn

QWEN3_MAPPINGS = (("input_layernorm", ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj")),
                  ("self_attn.v_proj", ("self_attn.o_proj",)),
                  ("post_attention_layernorm", ("mlp.gate_proj", "mlp.up_proj")),
                  ("mlp.up_proj", ("mlp.down_proj",)))


def fake_quant(w: torch.Tensor, group_size: int = 128, sym: bool = False) -> torch.Tensor:
    n, k = w.shape
    wg = w.float().view(n, k // group_size, group_size)
    s, z = quant_params(wg, 4, sym)
    q = torch.clamp(torch.round(wg / s[..., None]) + z[..., None], 0, 15)
    return ((q - z[..., None]) * s[..., None]).view(n, k)


@torch.no_grad()
def search_scale(x: torch.Tensor, weights: list[torch.Tensor], group_size: int = 128, n_grid: int = 20,
                 max_tokens: int = 4096) -> torch.Tensor:
    """Best per-input-channel scale for the linears ``weights`` (all reading ``x``)."""
    if x.shape[0] > max_tokens:
        idx = torch.linspace(0, x.shape[0] - 1, max_tokens, device=x.device).long()
        x = x[idx]
    x = x.float()
    x_mean = x.abs().mean(0)
    W = torch.cat([w.float() for w in weights], 0)
    n, k = W.shape
    wn = W.abs().view(n, k // group_size, group_size)
    wn = wn / wn.amax(-1, keepdim=True).clamp(min=1e-8)
    w_mean = wn.view(n, k).mean(0)
    ref = x @ W.t()
    best, best_s = float("inf"), torch.ones_like(x_mean)
    for i in range(n_grid):
        a = i / n_grid
        s = (x_mean.pow(a) / w_mean.pow(1 - a).clamp(min=1e-4)).clamp(min=1e-4)
        s = s / (s.max() * s.min()).sqrt()
        out = x @ (fake_quant(W * s[None], group_size) / s[None]).t()
        err = (ref - out).pow(2).mean().item()
        if err < best:
            best, best_s = err, s
    return best_s


@torch.no_grad()
def _fold(smooth: nn.Module, balance: list[nn.Linear], s: torch.Tensor):
    for lin in balance:
        lin.weight.data = (lin.weight.float() * s[None]).to(lin.weight.dtype)
    if isinstance(smooth, nn.Linear):               # previous linear's output channels
        smooth.weight.data = (smooth.weight.float() / s[:, None]).to(smooth.weight.dtype)
        if smooth.bias is not None:
            smooth.bias.data = (smooth.bias.float() / s).to(smooth.bias.dtype)
    else:                                           # RMSNorm / LayerNorm gain
        smooth.weight.data = (smooth.weight.float() / s).to(smooth.weight.dtype)
        if getattr(smooth, "bias", None) is not None:
            smooth.bias.data = (smooth.bias.float() / s).to(smooth.bias.dtype)


@torch.no_grad()
def awq_quantize_model(model: nn.Module, calib: Iterable[torch.Tensor], group_size: int = 128, n_grid: int = 20,
                       mappings=QWEN3_MAPPINGS, replace: bool = True, sym: bool = False) -> dict[str, Int4Weight]:
    walker = LayerWalker(model, calib)
    out: dict[str, Int4Weight] = {}
    for li, layer in enumerate(walker.layers):
        for smooth_name, bal_names in mappings:
            smooth = get_module(layer, smooth_name)
            bal = [get_module(layer, n) for n in bal_names]
            if isinstance(smooth, nn.Linear) and smooth.out_features != bal[0].in_features:
                continue                            # v_proj → o_proj under GQA: not foldable
            xs = []
            walker.collect_inputs(layer, bal_names[:1], lambda n: (lambda x: xs.append(x)))
            s = search_scale(torch.cat(xs, 0), [b.weight for b in bal], group_size, n_grid)
            _fold(smooth, bal, s.to(bal[0].weight.device))
        for name in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "self_attn.o_proj",
                     "mlp.gate_proj", "mlp.up_proj", "mlp.down_proj"):
            lin = get_module(layer, name)
            out[f"model.layers.{li}.{name}"] = quantize_rtn(lin.weight.detach(), group_size, sym)
            lin.weight.data = out[f"model.layers.{li}.{name}"].dequantize(lin.weight.dtype).to(lin.weight.device)
        walker.run_layer(layer, update=True)
    if replace:
        replace_with_int4(model, out)
    return out
