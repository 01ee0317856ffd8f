"""GPTQ W4A16: ``bits=4, group_size=128, desc_act=False``
(``GPTQModel/quantize_qwen3_4b_gptq.py:16-21``; ``LLM-Compressor/GPTQ/quantize_qwen3_4b_gptq.py:21-26``
with ``scheme="W4A16"``, ``ignore=["lm_head"]``).

Per linear: H = 2·XᵀX over the calibration inputs, dampened by ``damp``·mean(diag H); columns are
quantised left to right in blocks of 128 with the optimal-brain-surgeon error feedback through
the upper Cholesky factor of H⁻¹; group scale/zero are taken from the *updated* weights at each
group start (static groups, no act-order).  Hessian accumulation and the Cholesky run as GPU
matmuls / rocSOLVER calls through torch when the model is on the MI355X.
"""
from __future__ import annotations

import math
from typing import Iterable

import torch
import torch.nn as nn

from .calib import QWEN3_SEQUENTIAL, LayerWalker, set_module
from .int4 import Int4Linear, Int4Weight, from_parts, quant_params


class GPTQ:
    def __init__(self, lin: nn.Linear):
        self.lin = lin
        k = lin.in_features
        self.H = torch.zeros(k, k, dtype=torch.float32, device=lin.weight.device)
        self.n = 0

    def add_batch(self, x: torch.Tensor):
        x = x.reshape(-1, x.shape[-1]).float()
        m = x.shape[0]
        self.H *= self.n / (self.n + m)
        self.n += m
        x = x * math.sqrt(2.0 / self.n)
        self.H += x.t() @ x

    @torch.no_grad()
    def quantize(self, group_size: int = 128, sym: bool = False, damp: float = 0.01,
                 blocksize: int = 128) -> Int4Weight:
        W = self.lin.weight.detach().float().clone()
        n, k = W.shape
        H = self.H.clone()
        dead = torch.diag(H) == 0
        H[dead, dead] = 1.0
        W[:, dead] = 0.0
        H += damp * torch.mean(torch.diag(H)) * torch.eye(k, device=H.device)
        L = torch.linalg.cholesky(H)
        Hinv = torch.cholesky_inverse(L)
        Hinv = torch.linalg.cholesky(Hinv, upper=True)
        Q = torch.zeros(n, k, dtype=torch.int64, device=W.device)
        scales = torch.zeros(n, k // group_size, device=W.device)
        zeros = torch.zeros(n, k // group_size, device=W.device)
        for i1 in range(0, k, blocksize):
            i2 = min(i1 + blocksize, k)
            W1 = W[:, i1:i2].clone()
            Err1 = torch.zeros_like(W1)
            Hinv1 = Hinv[i1:i2, i1:i2]
            for i in range(i2 - i1):
                col = i1 + i
                if col % group_size == 0:
                    g = col // group_size
                    blockw = torch.cat([W1[:, i:], W[:, i2:]], 1)[:, :group_size]
                    s, z = quant_params(blockw, 4, sym)
                    scales[:, g], zeros[:, g] = s, z
                g = col // group_size
                s, z = scales[:, g], zeros[:, g]
                w = W1[:, i]
                q = torch.clamp(torch.round(w / s) + z, 0, 15)
                Q[:, col] = q.long()
                dq = (q - z) * s
                err = (w - dq) / Hinv1[i, i]
                W1[:, i:] -= err[:, None] @ Hinv1[i, i:][None, :]
                Err1[:, i] = err
            W[:, i2:] -= Err1 @ Hinv[i1:i2, i2:]
        return from_parts(Q, scales, zeros, group_size, sym)


@torch.no_grad()
def gptq_quantize_model(model: nn.Module, calib: Iterable[torch.Tensor], group_size: int = 128, sym: bool = False,
                        damp: float = 0.01, sequential=QWEN3_SEQUENTIAL, replace: bool = True) -> dict[str, Int4Weight]:
    """Quantise every decoder linear in place (``lm_head`` / embeddings untouched).  Returns
    ``{module path: Int4Weight}``; with ``replace`` the linears become :class:`Int4Linear`."""
    walker = LayerWalker(model, calib)
    out: dict[str, Int4Weight] = {}
    for li, layer in enumerate(walker.layers):
        for group in sequential:
            gq = {}

            def fn_for(name):
                def f(x):
                    gq[name].add_batch(x)
                return f
            from .calib import get_module
            for name in group:
                gq[name] = GPTQ(get_module(layer, name))
            walker.collect_inputs(layer, group, fn_for)
            for name in group:
                lin = get_module(layer, name)
                qw = gptq_quantize_one(gq[name], group_size, sym, damp)
                lin.weight.data = qw.dequantize(lin.weight.dtype).to(lin.weight.device)   # later groups see it
                out[f"model.layers.{li}.{name}"] = qw
                del gq[name]
        walker.run_layer(layer, update=True)
    if replace:
        replace_with_int4(model, out)
    return out


def gptq_quantize_one(g: GPTQ, group_size: int, sym: bool, damp: float) -> Int4Weight:
    try:
        return g.quantize(group_size, sym, damp)
    except torch.linalg.LinAlgError:            # not positive definite: more dampening
        return g.quantize(group_size, sym, damp * 10)


def replace_with_int4(model: nn.Module, weights: dict[str, Int4Weight]):
    from .calib import get_module
    for path, w in weights.items():
        lin = get_module(model, path)
        bias = getattr(lin, "bias", None)
        dev = lin.weight.device if hasattr(lin, "weight") else w.codes.device
        set_module(model, path, Int4Linear.from_weight(w.to(dev), bias))
