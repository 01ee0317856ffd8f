"""Multi-adapter LoRA serving: vLLM ``--enable-lora --lora-modules name1=dir1 name2=dir2``
(``Fine-Tuning/README.md:346-351``) — one frozen base model, several PEFT adapters, the adapter
chosen PER REQUEST by its ``model`` name, requests for different adapters (and the bare base)
batched together in the same decode step.

MI355X design: no per-adapter GEMM loop and no row sorting.  For every targeted projection the
adapters' LoRA factors are stacked once at load time:

    A_all [Σr, K]   (adapter a owns rows [o_a, o_a + r_a))
    B_all [N, Σr]   (the matching columns)

and on the GPU one segment kernel per projection (``csrc/kernels/mlora.hip``) computes, for every
row, only its own adapter's ``s_a·(x·A_aᵀ)·B_aᵀ`` — ``r_a·(K + N)`` MACs per row however many adapters
are loaded.  The portable form (CPU, odd ranks) computes ``y += ((x · A_allᵀ) ⊙ S[ids]) · B_allᵀ`` where ``S`` is a tiny
``[n_adapters + 1, Σr]`` table holding ``alpha_a / r_a`` on adapter a's columns (row 0 = the base,
all zeros) and ``ids`` the per-row adapter index.  That is the same low-rank K-slice the fused
training kernels use, segment-by-adapter through a column mask instead of a gather, so the step
has static shapes — it is captured in the decode hipGraph like everything else — and costs
``Σr·(K + N)`` MACs per row (≈1 % of the base GEMM for four r=16 adapters on Qwen3-8B).

``ids`` live in a device buffer owned by :class:`MultiLoraManager`: the serving engine writes a
slot's adapter index when it admits a request (decode rows = slots) and installs a per-token
index vector for packed prefill.
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn as nn


class MultiLoraSlot:
    """Stacked LoRA factors of every adapter for one projection."""

    def __init__(self, mgr: "MultiLoraManager", a_all: torch.Tensor, b_all: torch.Tensor, col_scale: torch.Tensor,
                 seg: list[tuple[int, int, float]] | None = None):
        self.mgr, self.A, self.B, self.col_scale = mgr, a_all, b_all, col_scale
        # per-adapter (offset, rank, scale) for the segment kernel (csrc/kernels/mlora.hip): each row
        # computes only its own adapter's rank-r_a term — cost independent of how many are loaded
        self.seg = None
        if seg is not None and a_all.is_cuda and all(r % 8 == 0 and r <= 64 and o % 8 == 0 for o, r, _ in seg) \
                and a_all.shape[0] % 8 == 0 and a_all.shape[1] % 8 == 0 and b_all.shape[0] % 8 == 0:
            import struct
            rows = [[o, r, struct.unpack("<i", struct.pack("<f", float(sc)))[0]] for o, r, sc in seg]
            self.seg = torch.tensor(rows, dtype=torch.int32, device=a_all.device)

    def delta(self, x: torch.Tensor) -> torch.Tensor:
        ids = self.mgr.row_ids(x.shape[0])
        xa = x.to(self.A.dtype) @ self.A.t()                              # [T, Σr]
        xa = xa * self.col_scale.index_select(0, ids)                    # zero foreign adapters' columns
        return xa @ self.B.t()                                           # [T, N]

    def apply_(self, x: torch.Tensor, y: torch.Tensor, c0: int = 0) -> torch.Tensor:
        if (self.seg is not None and x.dtype == torch.bfloat16 and y.dtype == torch.bfloat16 and x.stride(-1) == 1
                and y.stride(-1) == 1 and x.stride(0) % 8 == 0 and y.stride(0) % 8 == 0 and c0 % 8 == 0):
            from ..ops._native import native
            native().mlora_apply(x, self.A, self.B, self.mgr.row_ids(x.shape[0]), self.seg, y, c0)
            return y
        d = self.delta(x).to(y.dtype)
        if c0 == 0 and d.shape[1] == y.shape[1]:
            return y.add_(d)
        y[:, c0:c0 + d.shape[1]].add_(d)
        return y


def _read_adapter(directory: str) -> tuple[dict, dict[str, tuple[torch.Tensor, torch.Tensor]]]:
    from safetensors.torch import load_file
    with open(os.path.join(directory, "adapter_config.json")) as f:
        cfg = json.load(f)
    sd = load_file(os.path.join(directory, "adapter_model.safetensors"))
    mods: dict[str, dict] = {}
    for k, v in sd.items():
        name = k.removeprefix("base_model.model.")
        for tag in (".lora_A.", ".lora_B."):
            if tag in name:
                mod = name.split(tag)[0]
                mods.setdefault(mod, {})["A" if "A" in tag else "B"] = v
    out = {m: (d["A"], d["B"]) for m, d in mods.items() if "A" in d and "B" in d}
    return cfg, out


class MultiLoraManager:
    """Load several PEFT adapters next to a frozen base and attach a :class:`MultiLoraSlot` to
    every targeted projection (``module._mlora``).  Adapter 0 is the bare base model."""

    def __init__(self, model: nn.Module, adapters: dict[str, str], max_rows: int = 1 << 16):
        self.names = list(adapters)
        self.index = {n: i + 1 for i, n in enumerate(self.names)}      # 0 = base
        dev = next(model.parameters()).device
        loaded = {n: _read_adapter(d) for n, d in adapters.items()}
        modules = dict(model.named_modules())
        targets = sorted({m for _, mods in loaded.values() for m in mods})
        self.slots: dict[str, MultiLoraSlot] = {}
        dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
        for tname in targets:
            mod = modules.get(tname) or modules.get("model." + tname) or modules.get(tname.removeprefix("model."))
            if mod is None:
                raise KeyError(f"adapter target {tname!r} not found in the base model")
            leaf = getattr(mod, "base_layer", mod)
            K, N = leaf.in_features, leaf.out_features
            parts, cols, scales = [], [], []
            for n in self.names:
                cfg, mods = loaded[n]
                ab = mods.get(tname)
                r = 0 if ab is None else ab[0].shape[0]
                parts.append(ab)
                cols.append(r)
                scales.append(float(cfg.get("lora_alpha", r)) / max(1, int(cfg.get("r", r) or r)) if r else 0.0)
            R = sum(cols)
            a_all = torch.zeros(R, K, dtype=dtype, device=dev)
            b_all = torch.zeros(N, R, dtype=dtype, device=dev)
            col_scale = torch.zeros(len(self.names) + 1, R, dtype=dtype, device=dev)
            seg = [(0, 0, 0.0)]                     # adapter 0 = the bare base
            o = 0
            for i, (ab, r, s) in enumerate(zip(parts, cols, scales)):
                seg.append((o, r, s))
                if ab is None:
                    continue
                a_all[o:o + r] = ab[0].to(dev, dtype)
                b_all[:, o:o + r] = ab[1].to(dev, dtype)
                col_scale[i + 1, o:o + r] = s
                o += r
            slot = MultiLoraSlot(self, a_all, b_all, col_scale, seg)
            leaf._mlora = slot
            self.slots[tname] = slot
        self._buf = torch.zeros(max_rows, dtype=torch.long, device=dev)   # per-row adapter index
        self._ids = self._buf

    # ---- row → adapter mapping ---------------------------------------------------------
    def adapter_id(self, name: str | None, base_names=()) -> int:
        """``model`` field of a request → adapter index (0 = base); KeyError for unknown names."""
        if name is None or name in base_names:
            return 0
        return self.index[name]

    def row_ids(self, T: int) -> torch.Tensor:
        return self._ids[:T]

    def use_rows(self, ids: torch.Tensor | None):
        """Install a per-row index vector for the next forward (None: back to the slot buffer)."""
        self._ids = self._buf if ids is None else ids.to(self._buf.device, torch.long)

    def set_slot(self, slot: int, adapter: int):
        self._buf[slot] = adapter

    @property
    def slot_ids(self) -> torch.Tensor:
        return self._buf


def mlora_slot(m: nn.Module) -> MultiLoraSlot | None:
    return getattr(getattr(m, "base_layer", m), "_mlora", None)
