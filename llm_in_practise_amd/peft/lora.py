"""LoRA / QLoRA adaptation layer — PEFT-compatible, no peft import.

Reference surface:
  * ``LoraConfig(task_type=CAUSAL_LM, r, lora_alpha, lora_dropout, target_modules, bias="none")``
    (``Fine-Tuning/qwen3-8b-qlora.py:107-114``);
  * ``get_peft_model`` / ``print_trainable_parameters`` (``qwen3-8b-qlora-dist.py:124-132``);
  * ``prepare_model_for_kbit_training`` (``qwen3-8b-qlora.py:104``);
  * ``model.save_pretrained`` → ``adapter_model.safetensors`` + ``adapter_config.json``;
  * ``PeftModel.from_pretrained(base, dir)`` (``Fine-Tuning/inferences.py:25``);
  * ``merge_and_unload()`` (``Scripts/fine-tuning/02-merge-lora-adapter-and-model.py:32``).

Init follows PEFT [ext]: A ~ kaiming-uniform(a=√5), B = 0, scaling = alpha / r.
Adapter tensor names follow PEFT's on-disk convention
``base_model.model.<module path>.lora_{A,B}.weight``.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
import re
from typing import Iterable

import torch
import torch.nn as nn

from ..ops.linear import LoraBranch, fused_linear
from ..quant.nf4 import NF4Weight, dequantize_nf4, quantize_nf4


# ============================================================================ base layers
class Linear4bit(nn.Module):
    """Frozen NF4-quantised linear (the ``bnb.nn.Linear4bit`` role).  Quantised tensors are
    buffers so ``.to()`` / ``state_dict`` carry them."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False,
                 compute_dtype=torch.bfloat16, blocksize: int = 64):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.compute_dtype, self.blocksize = compute_dtype, blocksize
        self.register_buffer("codes", torch.zeros(0, dtype=torch.uint8))
        self.register_buffer("qabsmax", None)
        self.register_buffer("absmax", None)
        self.register_buffer("absmax2", None)
        self.register_buffer("offset", None)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=compute_dtype), requires_grad=False) if bias else None

    @classmethod
    def from_linear(cls, lin: nn.Linear, double_quant: bool = True, compute_dtype=torch.bfloat16,
                    device=None) -> "Linear4bit":
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, compute_dtype)
        w = lin.weight.detach()
        if device is not None:
            w = w.to(device)
        m.load_nf4(quantize_weight(w, double_quant, compute_dtype))
        if lin.bias is not None:
            m.bias.data = lin.bias.detach().to(device or lin.bias.device, compute_dtype)
        return m

    def load_nf4(self, q: NF4Weight):
        self.codes = q.codes
        self.absmax, self.qabsmax, self.absmax2, self.offset = q.absmax, q.qabsmax, q.absmax2, q.offset
        self.blocksize = q.blocksize

    @property
    def nf4(self) -> NF4Weight:
        c = self.__dict__.get("_nf4_cache")
        if c is None or c.codes is not self.codes:
            c = NF4Weight(self.codes, self.absmax, self.qabsmax, self.absmax2, self.offset,
                          (self.out_features, self.in_features), self.blocksize, self.compute_dtype)
            self.__dict__["_nf4_cache"] = c
        return c

    @property
    def weight(self):  # dequantised view for code that inspects ``.weight``
        return dequantize_nf4(self.nf4, self.compute_dtype)

    def forward(self, x):
        return fused_linear(x.to(self.compute_dtype), self.nf4, self.bias, (), training=self.training)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, nf4, blocksize={self.blocksize}"


def quantize_weight(w: torch.Tensor, double_quant: bool = True, compute_dtype=torch.bfloat16) -> NF4Weight:
    """Quantise with the HIP kernel when on the GPU, else the PyTorch reference."""
    from ..ops._native import use_native, native
    if use_native(w) and w.shape[1] % 64 == 0:
        codes, absmax = native().nf4_quantize(w.contiguous().to(torch.bfloat16), 64)
        q = NF4Weight(codes, absmax, None, None, None, tuple(w.shape), 64, compute_dtype)
        if double_quant:
            from ..quant.nf4 import double_quantize_absmax
            q = double_quantize_absmax(q)
        return q
    return quantize_nf4(w, 64, double_quant, compute_dtype)


# ============================================================================ LoRA layer
@dataclasses.dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: int = 16
    lora_dropout: float = 0.0
    target_modules: list[str] | str = dataclasses.field(default_factory=lambda: ["q_proj", "v_proj"])
    bias: str = "none"
    task_type: str = "CAUSAL_LM"
    modules_to_save: list[str] | None = None
    fan_in_fan_out: bool = False
    init_lora_weights: bool = True
    base_model_name_or_path: str | None = None
    inference_mode: bool = False
    peft_type: str = "LORA"

    @property
    def scaling(self) -> float:
        return self.lora_alpha / self.r

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        if isinstance(d["target_modules"], (set, tuple)):
            d["target_modules"] = sorted(d["target_modules"])
        return d


class TaskType:
    CAUSAL_LM = "CAUSAL_LM"
    SEQ_CLS = "SEQ_CLS"


class LoraLayer(nn.Module):
    """``base_layer`` + ``lora_A``/``lora_B``.  Forward is one fused GEMM (see ops.linear)."""

    def __init__(self, base_layer: nn.Module, r: int, alpha: int, dropout: float, init: bool = True):
        super().__init__()
        self.base_layer = base_layer
        in_f, out_f = _features(base_layer)
        dev = _module_device(base_layer)
        self.lora_A = nn.Linear(in_f, r, bias=False, device=dev, dtype=torch.float32)
        self.lora_B = nn.Linear(r, out_f, bias=False, device=dev, dtype=torch.float32)
        self.r, self.lora_alpha, self.lora_dropout = r, alpha, dropout
        self.scaling = alpha / r
        self.merged = False
        if init:
            nn.init.kaiming_uniform_(self.lora_A.weight, a=math.sqrt(5))
            nn.init.zeros_(self.lora_B.weight)
        for p in base_layer.parameters():
            p.requires_grad_(False)

    @property
    def in_features(self):
        return _features(self.base_layer)[0]

    @property
    def out_features(self):
        return _features(self.base_layer)[1]

    def branch(self, c0: int = 0) -> LoraBranch:
        return LoraBranch(self.lora_A.weight, self.lora_B.weight, self.scaling,
                          self.lora_dropout if self.training else 0.0, c0, c0 + self.out_features)

    def forward(self, x):
        base, bias = base_of(self.base_layer)
        cd = _compute_dtype(self.base_layer)
        branches = [] if self.merged else [self.branch()]
        return fused_linear(x.to(cd), base, bias, branches, training=self.training)

    @torch.no_grad()
    def merge(self) -> nn.Module:
        """W ← W + s·B·A (K19); QLoRA merges into a dequantised bf16 weight."""
        delta = (self.lora_B.weight.float() @ self.lora_A.weight.float()) * self.scaling
        bl = self.base_layer
        if isinstance(bl, Linear4bit):
            w = dequantize_nf4(bl.nf4, torch.float32) + delta.to(bl.codes.device)
            lin = nn.Linear(bl.in_features, bl.out_features, bias=bl.bias is not None,
                            device=bl.codes.device, dtype=bl.compute_dtype)
            lin.weight.copy_(w.to(bl.compute_dtype))
            if bl.bias is not None:
                lin.bias.copy_(bl.bias)
            return lin
        bl.weight.add_(delta.to(bl.weight.dtype))
        return bl


def _features(m: nn.Module) -> tuple[int, int]:
    return m.in_features, m.out_features


def _module_device(m: nn.Module):
    for t in list(m.parameters()) + list(m.buffers()):
        return t.device
    return torch.device("cpu")


def _compute_dtype(m: nn.Module):
    if isinstance(m, Linear4bit):
        return m.compute_dtype
    return m.weight.dtype


def base_of(m: nn.Module):
    """(base weight | NF4Weight, bias) of a plain projection module."""
    if isinstance(m, Linear4bit):
        return m.nf4, m.bias
    if isinstance(m, LoraLayer):
        return base_of(m.base_layer)
    return m.weight, m.bias


# ============================================================================ model-level API
def _match(name: str, targets) -> bool:
    if isinstance(targets, str):
        if targets == "all-linear":
            return not name.endswith("lm_head")
        return re.fullmatch(targets, name) is not None
    leaf = name.split(".")[-1]
    return leaf in targets


def inject_lora(model: nn.Module, config: LoraConfig) -> list[str]:
    names = []
    for name, mod in list(model.named_modules()):
        if isinstance(mod, (nn.Linear, Linear4bit)) and not isinstance(mod, LoraLayer) and _match(name, config.target_modules):
            if name.endswith("lora_A") or name.endswith("lora_B"):
                continue
            parent_name, _, leaf = name.rpartition(".")
            parent = model.get_submodule(parent_name) if parent_name else model
            setattr(parent, leaf, LoraLayer(mod, config.r, config.lora_alpha, config.lora_dropout,
                                            config.init_lora_weights))
            names.append(name)
    return names


class PeftModel(nn.Module):
    """Mirror of ``peft.PeftModel`` naming: ``peft_model.base_model.model`` is the wrapped
    model, so module paths (and therefore adapter keys) match PEFT's."""

    def __init__(self, model: nn.Module, config: LoraConfig):
        super().__init__()
        self.base_model = _LoraModel(model)
        self.peft_config = {"default": config}
        for p in model.parameters():
            p.requires_grad_(False)
        self.targets = inject_lora(model, config)
        for n, p in model.named_parameters():
            if "lora_" in n:
                p.requires_grad_(True)
        if config.modules_to_save:
            for n, p in model.named_parameters():
                if any(m in n for m in config.modules_to_save):
                    p.requires_grad_(True)

    @property
    def model(self) -> nn.Module:
        return self.base_model.model

    @property
    def config(self):
        return getattr(self.model, "config", None)

    def forward(self, *args, **kw):
        return self.model(*args, **kw)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.base_model.model, name)

    def get_nb_trainable_parameters(self) -> tuple[int, int]:
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        total = 0
        for m in self.modules():
            if isinstance(m, Linear4bit):
                total += m.in_features * m.out_features
            for p in m.parameters(recurse=False):
                total += p.numel()
        return trainable, total

    def print_trainable_parameters(self):
        t, a = self.get_nb_trainable_parameters()
        print(f"trainable params: {t:,d} || all params: {a:,d} || trainable%: {100 * t / max(a, 1):.4f}")

    # ------------------------------------------------------------------ adapter IO
    def adapter_state_dict(self) -> dict[str, torch.Tensor]:
        out = {}
        for n, p in self.model.named_parameters():
            if "lora_A" in n or "lora_B" in n or (self.peft_config["default"].modules_to_save and p.requires_grad):
                out[f"base_model.model.{n}"] = p.detach().to("cpu").contiguous()
        return out

    def save_pretrained(self, save_directory: str, safe_serialization: bool = True, **_):
        from safetensors.torch import save_file
        os.makedirs(save_directory, exist_ok=True)
        save_file(self.adapter_state_dict(), os.path.join(save_directory, "adapter_model.safetensors"),
                  metadata={"format": "pt"})
        cfg = self.peft_config["default"].to_dict()
        cfg["target_modules"] = sorted({t.split(".")[-1] for t in self.targets}) or cfg["target_modules"]
        with open(os.path.join(save_directory, "adapter_config.json"), "w") as f:
            json.dump(cfg, f, indent=2)

    def load_adapter(self, directory: str, strict: bool = True):
        from safetensors.torch import load_file
        sd = load_file(os.path.join(directory, "adapter_model.safetensors"))
        params = dict(self.model.named_parameters())
        missing = []
        for k, v in sd.items():
            name = k.removeprefix("base_model.model.")
            name = name.replace(".lora_A.default.", ".lora_A.").replace(".lora_B.default.", ".lora_B.")
            if name in params:
                with torch.no_grad():
                    params[name].copy_(v.to(params[name].dtype))
                    sh = getattr(params[name], "_lipa_shadow", None)
                    if sh is not None:           # optimizer-maintained bf16 shadow
                        sh.copy_(params[name])
            else:
                missing.append(k)
        if strict and missing:
            raise KeyError(f"adapter keys not in model: {missing[:5]}")

    @classmethod
    def from_pretrained(cls, model: nn.Module, directory: str, is_trainable: bool = False) -> "PeftModel":
        with open(os.path.join(directory, "adapter_config.json")) as f:
            cfgd = json.load(f)
        fields = {f.name for f in dataclasses.fields(LoraConfig)}
        cfg = LoraConfig(**{k: v for k, v in cfgd.items() if k in fields})
        pm = cls(model, cfg)
        pm.load_adapter(directory)
        if not is_trainable:
            for p in pm.parameters():
                p.requires_grad_(False)
            pm.eval()
        return pm

    @torch.no_grad()
    def merge_and_unload(self) -> nn.Module:
        model = self.model
        for name, mod in list(model.named_modules()):
            if isinstance(mod, LoraLayer):
                parent_name, _, leaf = name.rpartition(".")
                parent = model.get_submodule(parent_name) if parent_name else model
                setattr(parent, leaf, mod.merge())
        if hasattr(model, "invalidate_fusion"):
            model.invalidate_fusion()
        return model


class _LoraModel(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.model = model


def get_peft_model(model: nn.Module, config: LoraConfig) -> PeftModel:
    pm = PeftModel(model, config)
    if hasattr(model, "invalidate_fusion"):
        model.invalidate_fusion()
    return pm


def prepare_model_for_kbit_training(model: nn.Module, use_gradient_checkpointing: bool = True,
                                    gradient_checkpointing_kwargs: dict | None = None) -> nn.Module:
    """PEFT semantics [ext]: freeze everything, upcast non-quantised fp16/bf16 params (norms,
    embeddings) to fp32, enable input grads + gradient checkpointing.  On MI355X we keep
    norm/embedding weights in bf16 storage (frozen, read-only) — the upcast only exists in
    PEFT to stabilise fp16 training on small GPUs; numerics of the frozen forward are
    unchanged because our kernels accumulate in fp32."""
    for p in model.parameters():
        p.requires_grad_(False)
    if use_gradient_checkpointing and hasattr(model, "gradient_checkpointing_enable"):
        model.gradient_checkpointing_enable(gradient_checkpointing_kwargs)
    return model


def quantize_model_nf4(model: nn.Module, skip: Iterable[str] = ("lm_head", "lora_A", "lora_B"), double_quant: bool = True,
                       compute_dtype=torch.bfloat16) -> nn.Module:
    """Replace every ``nn.Linear`` (except ``skip``) by :class:`Linear4bit` — the
    ``from_pretrained(quantization_config=BitsAndBytesConfig(nf4))`` role."""
    for name, mod in list(model.named_modules()):
        if isinstance(mod, nn.Linear) and not any(name.endswith(s) for s in skip):
            parent_name, _, leaf = name.rpartition(".")
            parent = model.get_submodule(parent_name) if parent_name else model
            q = Linear4bit.from_linear(mod, double_quant, compute_dtype)
            setattr(parent, leaf, q)
            del mod
    if hasattr(model, "invalidate_fusion"):
        model.invalidate_fusion()
    return model
