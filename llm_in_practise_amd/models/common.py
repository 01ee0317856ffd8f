"""Shared model plumbing: fused projections, output container, KV cache."""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn

from ..ops.linear import LoraBranch, fused_linear
from ..peft.lora import Linear4bit, LoraLayer, base_of
from ..quant.int4 import Int4Linear, Int4Weight, int4_linear
from ..quant.nf4 import NF4Weight, concat_nf4


@dataclasses.dataclass
class CausalLMOutput:
    loss: torch.Tensor | None = None
    logits: torch.Tensor | None = None
    past_key_values: object | None = None
    hidden_states: torch.Tensor | None = None

    def __getitem__(self, i):
        return [v for v in (self.loss, self.logits) if v is not None][i]


def _leaf_linear(m: nn.Module) -> nn.Module:
    return m.base_layer if isinstance(m, LoraLayer) else m


def _out_features(m: nn.Module) -> int:
    return _leaf_linear(m).out_features


def _trainable_base(m: nn.Module) -> bool:
    leaf = _leaf_linear(m)
    return isinstance(leaf, nn.Linear) and leaf.weight.requires_grad


class FusedProjection:
    """Row-concatenation of projections that share one input (q|k|v, gate|up).

    The concatenated base replaces the parts' storage (each part's buffers / weight become
    views into it), so fusion costs no extra HBM.  LoRA branches keep their own A/B and
    address their column range of the fused output.  Not used when a base weight is
    trainable (full fine-tune) — then each projection runs on its own.
    """

    def __init__(self, mods: list[nn.Module]):
        self.mods = mods
        leaves = [_leaf_linear(m) for m in mods]
        self.splits = [_out_features(m) for m in mods]
        if all(isinstance(l, Linear4bit) for l in leaves):
            parts = [l.nf4 for l in leaves]
            fused = concat_nf4(parts)
            self.base: NF4Weight | torch.Tensor = fused
            r0, b0 = 0, 0
            for l in leaves:                      # re-point parts at views of the fused storage
                n = l.out_features
                nblk = n * l.in_features // l.blocksize
                l.codes = fused.codes[r0:r0 + n]
                if fused.double_quant:
                    g0, ng = b0 // 256, nblk // 256
                    l.qabsmax = fused.qabsmax[b0:b0 + nblk]
                    l.absmax2 = fused.absmax2[g0:g0 + ng]
                    l.offset = fused.offset[g0:g0 + ng]
                else:
                    l.absmax = fused.absmax[b0:b0 + nblk]
                r0 += n
                b0 += nblk
            biases = [l.bias for l in leaves]
        elif all(isinstance(l, Int4Linear) for l in leaves):   # W4A16 (GPTQ / AWQ / RTN): concat along N
            codes = torch.cat([l.codes for l in leaves], 0)
            scales = torch.cat([l.scales for l in leaves], 0)
            zeros = torch.cat([l.zeros for l in leaves], 0)
            self.base = Int4Weight(codes, scales, zeros, (codes.shape[0], leaves[0].in_features),
                                   leaves[0].group_size, leaves[0].sym)
            r0 = 0
            for l in leaves:
                n = l.out_features
                l.load(Int4Weight(codes[r0:r0 + n], scales[r0:r0 + n], zeros[r0:r0 + n], (n, l.in_features),
                                  l.group_size, l.sym))
                r0 += n
            biases = [l.bias for l in leaves]
        else:
            w = torch.cat([l.weight.detach() for l in leaves], 0)
            self.base = w
            r0 = 0
            for l in leaves:
                n = l.out_features
                l.weight = nn.Parameter(w[r0:r0 + n], requires_grad=False)
                r0 += n
            biases = [l.bias for l in leaves]
        self.bias = None
        if any(b is not None for b in biases):
            self.bias = torch.cat([b.detach() if b is not None else torch.zeros(n, dtype=self.dtype, device=self.device)
                                   for b, n in zip(biases, self.splits)])

    @property
    def dtype(self):
        return self.base.dtype

    @property
    def device(self):
        return self.base.device

    def branches(self, training: bool) -> list[LoraBranch]:
        out, c0 = [], 0
        for m, n in zip(self.mods, self.splits):
            if isinstance(m, LoraLayer) and not m.merged:
                br = m.branch(c0)
                if not training:
                    br.dropout = 0.0
                out.append(br)
            c0 += n
        return out

    def __call__(self, x, residual=None, training: bool = True):
        if isinstance(self.base, Int4Weight):
            y = int4_linear(x, self.base, self.bias, residual)
            for br in self.branches(False):       # inference-only base: unmerged adapters as plain low-rank adds
                y2 = y.view(-1, y.shape[-1])
                y2[:, br.c0:br.c1] += ((x.reshape(-1, x.shape[-1]) @ br.a.t().to(x.dtype)) @ br.b.t().to(x.dtype)) * br.scaling
            return _apply_multi_lora(self.mods, self.splits, x, y)
        y = fused_linear(x, self.base, self.bias, self.branches(training), residual, training)
        return _apply_multi_lora(self.mods, self.splits, x, y)


def _apply_multi_lora(mods, splits, x, y):
    """Per-request adapters of multi-LoRA serving (``peft/multi_lora.py``): y[:, c0:c1] += the
    row-masked stacked low-rank term of each projection that carries adapters."""
    slots = [getattr(_leaf_linear(m), "_mlora", None) for m in mods]
    if not any(s is not None for s in slots):
        return y
    x2, y2 = x.reshape(-1, x.shape[-1]), y.view(-1, y.shape[-1])
    c0 = 0
    for s, n in zip(slots, splits):
        if s is not None:
            s.apply_(x2, y2, c0)
        c0 += n
    return y


def project(mods: list[nn.Module], x: torch.Tensor, residual: torch.Tensor | None = None,
            training: bool = True, fused: FusedProjection | None = None) -> torch.Tensor:
    """Run projections that share input ``x`` and concatenate their outputs."""
    if fused is not None:
        return fused(x, residual, training)
    if len(mods) == 1:
        m = mods[0]
        if isinstance(m, Int4Linear):            # o_proj / down_proj of a W4A16 model: residual in the epilogue
            y = int4_linear(x.to(torch.bfloat16) if x.is_cuda else x, m.int4, m.bias, residual)
            return _apply_multi_lora(mods, [m.out_features], x, y)
        if _trainable_base(m) or not isinstance(_leaf_linear(m), (nn.Linear, Linear4bit)):
            y = m(x)
            y = _apply_multi_lora(mods, [y.shape[-1]], x, y)
            return y if residual is None else y + residual
        base, bias = base_of(m)
        br = [m.branch()] if isinstance(m, LoraLayer) and not m.merged else []
        if br and not training:
            br[0].dropout = 0.0
        cd = base.dtype if isinstance(base, torch.Tensor) else base.dtype
        y = fused_linear(x.to(cd), base, bias, br, residual, training)
        return _apply_multi_lora(mods, [_out_features(m)], x, y)
    ys = [project([m], x, None, training) for m in mods]
    y = torch.cat(ys, -1)
    return y if residual is None else y + residual


def can_fuse(mods: list[nn.Module]) -> bool:
    leaves = [_leaf_linear(m) for m in mods]
    if any(_trainable_base(m) for m in mods):
        return False
    if all(isinstance(l, Linear4bit) for l in leaves):
        k = leaves[0].in_features
        return all(l.in_features == k and (l.out_features * l.in_features // l.blocksize) % 256 == 0 for l in leaves)
    if all(isinstance(l, Int4Linear) for l in leaves):
        return len({(l.in_features, l.group_size, l.sym) for l in leaves}) == 1
    if all(isinstance(l, nn.Linear) for l in leaves):
        return len({l.in_features for l in leaves}) == 1 and len({l.weight.dtype for l in leaves}) == 1
    return False


class PackedPrefill:
    """Prefill of several prompts packed back to back — ``[1, T]`` tokens, no padding — straight
    into their KV-cache slots (the serving engine's admission path).

    Every token-wise op (projections, norms, SwiGLU: nearly all prefill FLOPs) runs on the
    packed tokens only; attention scatters q/k/v into a right-padded ``[B, S]`` view for the
    flash kernel (causal, per-row ``kv_lens``) and gathers the valid rows back, and each
    layer's K/V rows are written into the cache slots with one indexed copy.  Against padding
    every prompt to the longest one this removes the padded GEMM work (≈ 40 % on chat-length
    prompts) and the scratch-cache → slot copy."""

    def __init__(self, cache: "KVCache", slots: list[int], lens: list[int], device):
        self.cache, self.B, self.S = cache, len(lens), max(lens)
        self.len, self.pos = 0, None              # KVCache duck-typing: a prefill from position 0
        tb = torch.cat([torch.full((n,), b, dtype=torch.long) for b, n in enumerate(lens)])
        tp = torch.cat([torch.arange(n, dtype=torch.long) for n in lens])
        sl = torch.tensor(slots, dtype=torch.long)
        self.positions = tp.to(device)[None]
        self.pad_idx = (tb * self.S + tp).to(device)
        self.cache_idx = (sl[tb] * cache.max_len + tp).to(device)
        self.kv_lens = torch.tensor(lens, dtype=torch.int32, device=device)
        self.last = (torch.cumsum(torch.tensor(lens), 0) - 1).to(device)

    def attend(self, layer: int, q, k, v, hq: int, hkv: int, d: int, attention_fn):
        self.cache.k[layer].view(-1, hkv * d).index_copy_(0, self.cache_idx, k)
        self.cache.v[layer].view(-1, hkv * d).index_copy_(0, self.cache_idx, v)
        if self.B == 1:
            return attention_fn(q, k, v, 1, self.S, hq, hkv, d, causal=True, kv_lens=None)
        n = self.B * self.S

        def pad(t):
            out = t.new_zeros(n, t.shape[1])
            return out.index_copy_(0, self.pad_idx, t)
        o = attention_fn(pad(q), pad(k), pad(v), self.B, self.S, hq, hkv, d, causal=True, kv_lens=self.kv_lens)
        return o.index_select(0, self.pad_idx)


class KVCache:
    """Contiguous pre-allocated KV cache ``[B, Smax, Hkv*D]`` per layer (K17).

    Prefill writes a uniform prefix (``update``; rows may be right-padded, their valid lengths
    live in ``lens``); decode appends one token per row at its own position ``pos[b]``
    (``write_rows``), so a batch of prompts of different lengths decodes without re-padding.
    ``pos`` is a device tensor, so a decode step has no host sync (hipGraph-capturable)."""

    def __init__(self, n_layers: int, batch: int, max_len: int, hkv: int, d: int, dtype, device):
        self.k = [torch.zeros(batch, max_len, hkv * d, dtype=dtype, device=device) for _ in range(n_layers)]
        self.v = [torch.zeros(batch, max_len, hkv * d, dtype=dtype, device=device) for _ in range(n_layers)]
        self.len = 0
        self.max_len = max_len
        self.batch = batch
        self.pos: torch.Tensor | None = None      # [B] int64 next write position (decode mode)
        self._rows = torch.arange(batch, device=device)

    def update(self, layer: int, k: torch.Tensor, v: torch.Tensor, start: int):
        """k/v [B, s, Hkv*D] written at ``start``; returns views up to start+s."""
        s = k.shape[1]
        self.k[layer][:, start:start + s] = k
        self.v[layer][:, start:start + s] = v
        return self.k[layer][:, :start + s], self.v[layer][:, :start + s]

    def write_rows(self, layer: int, k: torch.Tensor, v: torch.Tensor):
        """k/v [B, Hkv*D] written at row-specific positions ``pos``."""
        self.k[layer][self._rows, self.pos] = k
        self.v[layer][self._rows, self.pos] = v

    def head_rows(self, n: int) -> "KVCache":
        """View of the first ``n`` rows sharing storage (and ``pos``) with this cache — the serving
        engine decodes only up to its highest occupied slot."""
        if n == self.batch:
            return self
        v = KVCache.__new__(KVCache)
        v.k = [t[:n] for t in self.k]
        v.v = [t[:n] for t in self.v]
        v.len, v.max_len, v.batch = self.len, self.max_len, n
        v.pos = self.pos[:n] if self.pos is not None else None
        v._rows = self._rows[:n]
        return v

    def start_decode(self, lens: torch.Tensor):
        self.pos = lens.to(torch.long).clone()

    def get_seq_length(self) -> int:
        return self.len
