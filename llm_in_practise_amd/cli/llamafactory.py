"""``llamafactory-cli train | export | webchat <yaml>`` equivalents.

Reference: ``Fine-Tuning/LLaMA-Factory/README.md:97-246`` and
``deepseek-r1-0528-qwen3_lora_sft.yaml`` — a YAML recipe with ``stage: sft``,
``finetuning_type: lora``, ``lora_target: all``, optional ``quantization_bit: 4``,
``cutoff_len``, ``template``, Trainer-style hyper-parameters, and ``export`` = merge.

The reference YAML is malformed (``dataset:`` given a scalar followed by list items): strict
YAML folds it into one plain scalar ``"a - b - c"``, which the loader splits back into the
intended list (and a line parser takes over for YAML that does not parse at all), so the shipped
recipe runs as written.  Unsupported keys are reported, not silently
applied (``packing``, ``enable_thinking``, ``flash_attn`` are accepted no-ops: attention is
always the fused gfx950 kernel).
"""
from __future__ import annotations

import json
import os
import re
import sys

import torch

LF_IGNORED = {"do_train", "overwrite_cache", "overwrite_output_dir", "plot_loss", "flash_attn", "packing",
              "enable_thinking", "preprocessing_num_workers", "ddp_timeout", "report_to", "trust_remote_code",
              "val_size", "eval_strategy", "eval_steps", "per_device_eval_batch_size", "dataloader_num_workers",
              "quantization_method", "double_quantization", "infer_backend", "export_size", "export_device",
              "export_legacy_format", "resume_from_checkpoint", "template"}


def load_lf_yaml(path: str) -> dict:
    import yaml
    text = open(path, encoding="utf-8").read()
    try:
        d = yaml.safe_load(text)
        if isinstance(d, dict):
            # strict YAML folds the reference's "dataset: a\n  - b\n  - c" into the plain scalar
            # "a - b - c": split it back into the intended list
            for k in ("dataset", "eval_dataset"):
                if isinstance(d.get(k), str):
                    d[k] = [t.strip() for part in re.split(r"\s+-\s+", d[k]) for t in part.split(",") if t.strip()]
            return d
    except yaml.YAMLError:
        pass
    # tolerant line parser: "key: value  # comment" and "  - item" continuation lines
    out, last = {}, None
    for raw in text.splitlines():
        line = re.sub(r"\s+#.*$", "", raw).rstrip()
        if not line.strip() or line.lstrip().startswith("#"):
            continue
        m = re.match(r"^\s*-\s*(.+)$", line)
        if m and last is not None:
            cur = out[last]
            out[last] = (cur if isinstance(cur, list) else ([cur] if cur not in (None, "") else [])) + [m.group(1)]
            continue
        m = re.match(r"^([A-Za-z_][\w.]*)\s*:\s*(.*)$", line)
        if m:
            last = m.group(1)
            out[last] = yaml.safe_load(m.group(2)) if m.group(2) else None
    return out


def _alpaca_to_sc(rec: dict) -> dict:
    """Alpaca (instruction / input / output) → the self-cognition schema the SFT pipeline takes."""
    if "query" in rec:
        return rec
    q = rec.get("instruction", "")
    if rec.get("input"):
        q = f"{q}\n{rec['input']}"
    return {"query": q, "response": rec.get("output", "")}


def resolve_datasets(names, dataset_dir: str) -> list[dict]:
    from ..train.data import load_records
    if isinstance(names, str):
        names = [n.strip() for n in names.split(",") if n.strip()]
    info = {}
    ip = os.path.join(dataset_dir, "dataset_info.json")
    if os.path.exists(ip):
        info = json.load(open(ip, encoding="utf-8"))
    recs = []
    for n in names or []:
        cands = [n, os.path.join(dataset_dir, n)]
        if n in info and "file_name" in info[n]:
            cands.insert(0, os.path.join(dataset_dir, info[n]["file_name"]))
        cands += [os.path.join(dataset_dir, n + ext) for ext in (".json", ".jsonl")]
        path = next((c for c in cands if os.path.isfile(c)), None)
        if path is None:
            raise FileNotFoundError(f"dataset {n!r} not found locally (looked in {dataset_dir}; no hub access)")
        recs += [_alpaca_to_sc(r) for r in load_records(path)]
    return recs


def lf_train(cfg: dict, tokenizer: str | None = None):
    from ..models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from ..parallel import dist as D
    from ..peft.lora import LoraConfig, get_peft_model, prepare_model_for_kbit_training, quantize_model_nf4
    from ..train.data import DEEPSEEK_R1_SYSTEM, QWEN3_SYSTEM, SFTDataset, load_tokenizer
    from ..train.trainer import Trainer, TrainingArguments
    unknown = sorted(k for k in cfg if k not in LF_IGNORED and k not in LF_KEYS)
    if unknown:
        print(f"[lipa lf] ignoring unsupported keys: {unknown}", file=sys.stderr)
    if cfg.get("stage", "sft") != "sft":
        raise NotImplementedError("only stage: sft (the reference recipe)")
    ftype = cfg.get("finetuning_type", "lora")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        D.init_distributed(timeout_s=1800)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    path = str(cfg["model_name_or_path"])
    dtype = torch.bfloat16 if (cfg.get("bf16") or dev.type == "cuda") else torch.float32
    if path.startswith("random:"):
        model = Qwen3ForCausalLM.from_config(qwen3_config(path[7:]), dtype=dtype, device=dev)
    else:
        rs = cfg.get("rope_scaling")
        model = Qwen3ForCausalLM.from_pretrained(path, dtype=dtype, device=dev,
                                                 rope_scaling="keep" if rs in (None, "yarn") else rs)
    q4 = int(cfg.get("quantization_bit") or 0) == 4
    if q4:
        quantize_model_nf4(model)
        model = prepare_model_for_kbit_training(model, use_gradient_checkpointing=False)
    if ftype == "lora":
        r = int(cfg.get("lora_rank", 8))
        tgt = cfg.get("lora_target", "all")
        targets = "all-linear" if tgt == "all" else [t.strip() for t in str(tgt).split(",")]
        model = get_peft_model(model, LoraConfig(r=r, lora_alpha=int(cfg.get("lora_alpha", 2 * r)),
                                                 lora_dropout=float(cfg.get("lora_dropout", 0.0)),
                                                 target_modules=targets, task_type="CAUSAL_LM"))
        if D.is_main():
            model.print_trainable_parameters()
        model.fuse_projections()
    elif ftype != "full":
        raise NotImplementedError(f"finetuning_type {ftype!r}")
    tok = load_tokenizer(tokenizer or (path if not path.startswith("random:") else "bytes"))
    system = DEEPSEEK_R1_SYSTEM if str(cfg.get("template", "")).startswith("deepseek") else QWEN3_SYSTEM
    recs = resolve_datasets(cfg.get("dataset"), cfg.get("dataset_dir", "data"))
    if cfg.get("max_samples"):
        recs = recs[:int(cfg["max_samples"])]
    ds = SFTDataset(recs, tok, int(cfg.get("cutoff_len", 2048)), padding="longest", label_mode="assistant",
                    system=system)
    args = TrainingArguments(
        output_dir=cfg.get("output_dir", "finetuned/lf"),
        per_device_train_batch_size=int(cfg.get("per_device_train_batch_size", 1)),
        gradient_accumulation_steps=int(cfg.get("gradient_accumulation_steps", 8)),
        num_train_epochs=float(cfg.get("num_train_epochs", 3.0)), max_steps=int(cfg.get("max_steps", -1)),
        learning_rate=float(cfg.get("learning_rate", 1e-4)), lr_scheduler_type=cfg.get("lr_scheduler_type", "cosine"),
        warmup_ratio=float(cfg.get("warmup_ratio", 0.0)), warmup_steps=int(cfg.get("warmup_steps", 0)),
        logging_steps=int(cfg.get("logging_steps", 10)), save_steps=int(cfg.get("save_steps", 500)),
        bf16=bool(cfg.get("bf16", dev.type == "cuda")), fp16=bool(cfg.get("fp16", False)),
        optim=cfg.get("optim", "adamw_torch"), report_to=[], remove_unused_columns=False,
        gradient_checkpointing=bool(cfg.get("gradient_checkpointing", False)),
        deepspeed=cfg.get("deepspeed"), seed=int(cfg.get("seed", 42)))
    tr = Trainer(model, args, train_dataset=ds, tokenizer=tok)
    out = tr.train()
    tr.save_model(args.output_dir)
    tr.save_metrics("train", out.metrics)
    tr.save_state()
    return out


LF_KEYS = {"model_name_or_path", "stage", "finetuning_type", "lora_target", "lora_rank", "lora_alpha",
           "lora_dropout", "quantization_bit", "dataset", "dataset_dir", "max_samples", "cutoff_len", "output_dir",
           "logging_steps", "save_steps", "per_device_train_batch_size", "gradient_accumulation_steps",
           "learning_rate", "num_train_epochs", "max_steps", "lr_scheduler_type", "warmup_ratio", "warmup_steps",
           "bf16", "fp16", "optim", "gradient_checkpointing", "deepspeed", "seed", "rope_scaling",
           "adapter_name_or_path", "export_dir"}


def lf_export(cfg: dict, tokenizer: str | None = None):
    """``llamafactory-cli export``: merge ``adapter_name_or_path`` into the base and save to ``export_dir``."""
    from ..models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from ..peft.lora import PeftModel
    path = str(cfg["model_name_or_path"])
    if path.startswith("random:"):
        base = Qwen3ForCausalLM.from_config(qwen3_config(path[7:]), dtype=torch.float32)
    else:
        base = Qwen3ForCausalLM.from_pretrained(path, dtype=torch.bfloat16)
    merged = PeftModel.from_pretrained(base, cfg["adapter_name_or_path"]).merge_and_unload()
    merged.save_pretrained(cfg["export_dir"])
    tp = tokenizer or (path if not path.startswith("random:") else None)
    if tp and os.path.exists(os.path.join(tp, "tokenizer.json")):
        from ..train.data import load_tokenizer
        load_tokenizer(tp).save_pretrained(cfg["export_dir"])
    return cfg["export_dir"]
