"""Quantised checkpoint IO (SURVEY.md F1-F4, §5.4 "Merge/quant" row).

``save_quantized`` writes an HF-layout directory: ``config.json`` (model config +
``quantization_config``), ``model.safetensors`` with the non-quantised tensors in bf16 and each
quantised linear in the chosen format's tensor names:

* ``compressed-tensors`` (default; what llm-compressor ``oneshot`` emits and what the reference
  serves with vLLM ``--quantization compressed-tensors``,
  ``Deployment/litellm-proxy/docker-compose-router-lb.yaml:81-89``);
* ``gptq`` (GPTQModel ``model.save``, ``GPTQModel/quantize_qwen3_4b_gptq.py:45-48``);
* ``awq`` (AutoAWQ GEMM / ``quantization_format="awq"``, ``Quantization/README.md:139-156``).

``load_quantized`` reads any of the three back into a model whose linears are
:class:`~llm_in_practise_amd.quant.int4.Int4Linear` (MFMA GEMM for prefill, GEMV for decode).
"""
from __future__ import annotations

import json
import os

import torch

from .calib import get_module, set_module
from .int4 import (Int4Linear, Int4Weight, from_awq, from_compressed_tensors, from_gptq, to_awq,
                   to_compressed_tensors, to_gptq)


def _quant_config(fmt: str, group_size: int, sym: bool, ignore=("lm_head",)) -> dict:
    if fmt == "compressed-tensors":
        return {"quant_method": "compressed-tensors", "format": "pack-quantized",
                "config_groups": {"group_0": {"targets": ["Linear"],
                                              "weights": {"num_bits": 4, "type": "int", "symmetric": sym,
                                                          "group_size": group_size, "strategy": "group"},
                                              "input_activations": None}},
                "ignore": list(ignore)}
    if fmt == "gptq":
        return {"quant_method": "gptq", "bits": 4, "group_size": group_size, "desc_act": False, "sym": sym,
                "checkpoint_format": "gptq"}
    if fmt == "awq":
        return {"quant_method": "awq", "bits": 4, "group_size": group_size, "zero_point": not sym, "version": "gemm"}
    raise ValueError(fmt)


def save_quantized(model, out_dir: str, fmt: str = "compressed-tensors", tokenizer=None):
    from safetensors.torch import save_file
    os.makedirs(out_dir, exist_ok=True)
    sd, gs, sym = {}, 128, False
    qpaths = set()
    for name, mod in model.named_modules():
        if isinstance(mod, Int4Linear):
            w = mod.int4
            gs, sym = w.group_size, w.sym
            qpaths.add(name)
            tens = {"compressed-tensors": to_compressed_tensors, "gptq": to_gptq, "awq": to_awq}[fmt](w)
            for k, v in tens.items():
                sd[f"{name}.{k}"] = v.contiguous()
            if mod.bias is not None:
                sd[f"{name}.bias"] = mod.bias.detach().cpu().to(torch.bfloat16)
    for k, v in model.state_dict().items():
        mod_path = k.rsplit(".", 1)[0]
        if mod_path in qpaths or "inv_freq" in k:
            continue
        sd[k] = v.detach().cpu().contiguous()
    cfg = getattr(model, "config", None)
    if cfg is not None and getattr(cfg, "tie_word_embeddings", False):
        sd.pop("lm_head.weight", None)
    save_file(sd, os.path.join(out_dir, "model.safetensors"), metadata={"format": "pt"})
    d = cfg.to_dict() if cfg is not None else {}
    d["torch_dtype"] = "bfloat16"
    d["quantization_config"] = _quant_config(fmt, gs, sym)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(d, f, indent=2)
    if tokenizer is not None and hasattr(tokenizer, "save_pretrained"):
        tokenizer.save_pretrained(out_dir)
    return out_dir


def _detect(qc: dict):
    m = qc.get("quant_method")
    if m == "compressed-tensors":
        w = next(iter(qc["config_groups"].values()))["weights"]
        return "compressed-tensors", int(w["group_size"]), bool(w.get("symmetric", False))
    if m == "gptq":
        return "gptq", int(qc.get("group_size", 128)), bool(qc.get("sym", True))
    if m == "awq":
        return "awq", int(qc.get("group_size", 128)), not bool(qc.get("zero_point", True))
    raise ValueError(f"unsupported quant_method {m}")


def load_quantized(path: str, device=None, dtype=torch.bfloat16):
    from safetensors import safe_open

    from ..models.qwen3 import Qwen3Config, Qwen3ForCausalLM
    from ..ops import reference as ref
    with open(os.path.join(path, "config.json")) as f:
        d = json.load(f)
    fmt, gs, sym = _detect(d["quantization_config"])
    cfg = Qwen3Config.from_dict(d)
    with torch.device("meta"):
        m = Qwen3ForCausalLM(cfg)
    m.to_empty(device=device or "cpu")
    m.to(dtype)
    sd = {}
    for fn in sorted(f for f in os.listdir(path) if f.endswith(".safetensors")):
        with safe_open(os.path.join(path, fn), framework="pt", device="cpu") as fh:
            for k in fh.keys():
                sd[k] = fh.get_tensor(k)
    marker = {"compressed-tensors": ".weight_packed", "gptq": ".qweight", "awq": ".qweight"}[fmt]
    qpaths = [k[: -len(marker)] for k in sd if k.endswith(marker)]
    for p in qpaths:
        pre = p + "."
        tens = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        if fmt == "compressed-tensors":
            w = from_compressed_tensors(tens, gs, sym)
        elif fmt == "gptq":
            w = from_gptq(tens, gs, sym)
        else:
            w = from_awq(tens, gs)
        set_module(m, p, Int4Linear.from_weight(w.to(device or "cpu"), tens.get("bias")))
        for k in list(tens):
            sd.pop(pre + k, None)
    m.load_hf_state_dict(sd)
    inv, af = ref.rope_inv_freq(cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
    m.model.inv_freq = inv.to(device or "cpu")
    m.model.attn_factor = af
    if cfg.tie_word_embeddings:
        m.lm_head.weight = m.model.embed_tokens.weight
    return m.eval()
