"""Layer-by-layer calibration driver shared by GPTQ and AWQ.

The reference calls ``model.quantize(calib)`` (GPTQModel, ``GPTQModel/quantize_qwen3_4b_gptq.py:42``)
or ``oneshot(model, recipe, dataset, num_calibration_samples=128, max_seq_length=2048)``
(llm-compressor, ``LLM-Compressor/AWQ/quantize_qwen3_4b_awq.py:45-58``).  Both walk the decoder
layer by layer: the calibration hidden states enter layer i, its linears' input statistics are
gathered, the layer is quantised, and its (now quantised) output becomes layer i+1's input — so
the whole model never needs more than one layer's activations at a time.  This module does that
walk for our decoder models (Qwen3 family) and exposes per-linear input taps.
"""
from __future__ import annotations

from typing import Callable, Iterable

import torch
import torch.nn as nn

from ..ops.linear import fused_linear

# quantisation order inside a decoder layer ("true sequential"): each group's inputs are taken
# after the previous groups were quantised
QWEN3_SEQUENTIAL = (("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"), ("self_attn.o_proj",),
                    ("mlp.gate_proj", "mlp.up_proj"), ("mlp.down_proj",))


class Tap(nn.Module):
    """Transparent wrapper that hands every input of a linear to ``fn`` (``project()`` calls
    non-``nn.Linear`` leaves through ``__call__``, so the tap sees the real activations)."""

    def __init__(self, lin: nn.Linear, fn: Callable[[torch.Tensor], None]):
        super().__init__()
        self.lin, self.fn = lin, fn
        self.in_features, self.out_features = lin.in_features, lin.out_features

    def forward(self, x):
        self.fn(x.detach().reshape(-1, x.shape[-1]))
        w = self.lin.weight
        return fused_linear(x.to(w.dtype), w, self.lin.bias, (), None, False)


def get_module(root: nn.Module, path: str) -> nn.Module:
    m = root
    for p in path.split("."):
        m = getattr(m, p)
    return m


def set_module(root: nn.Module, path: str, new: nn.Module):
    parent, _, leaf = path.rpartition(".")
    setattr(get_module(root, parent) if parent else root, leaf, new)


class LayerWalker:
    """Iterates the decoder layers of a Qwen3-style model with calibration activations."""

    def __init__(self, model: nn.Module, calib: Iterable[torch.Tensor]):
        self.model = model
        self.inner = model.model
        self.samples = []
        dev = next(model.parameters()).device
        with torch.no_grad():
            for ids in calib:
                ids = ids.to(dev)
                if ids.dim() == 1:
                    ids = ids[None]
                B, S = ids.shape
                pos = torch.arange(S, device=dev).expand(B, S)
                cos, sin = self.inner.rope(pos)
                x = self.inner.embed_tokens(ids).reshape(B * S, -1)
                self.samples.append([x, cos, sin, B, S])

    @property
    def layers(self):
        return self.inner.layers

    @torch.no_grad()
    def run_layer(self, layer: nn.Module, update: bool = False):
        """Forward every calibration sample through ``layer``; with ``update`` the outputs
        replace the stored inputs (advance to the next layer)."""
        for s in self.samples:
            y = layer(s[0], s[1], s[2], s[3], s[4])
            if update:
                s[0] = y

    @torch.no_grad()
    def collect_inputs(self, layer: nn.Module, names: Iterable[str], fn_for: Callable[[str], Callable]):
        names = list(names)
        origs = {n: get_module(layer, n) for n in names}
        try:
            for n, m in origs.items():
                set_module(layer, n, Tap(m, fn_for(n)))
            self.run_layer(layer)
        finally:
            for n, m in origs.items():
                set_module(layer, n, m)
        return origs
