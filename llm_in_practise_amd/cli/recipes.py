"""Fine-tuning presets = the reference scripts' hard-coded constants (SURVEY.md §2.1 Track E).

Each preset pins model family, quantisation, LoRA config, TrainingArguments and the SFT data
pipeline variant of one reference script, so ``lipa finetune --preset <name>`` reproduces it.
"""
from __future__ import annotations

import dataclasses

from ..train.data import DEEPSEEK_R1_SYSTEM, QWEN3_SYSTEM


@dataclasses.dataclass
class FinetunePreset:
    name: str
    source: str                               # reference script (file:lines)
    model: str                                # Qwen3 preset for --random-init, or documentation
    quant: str | None                         # None | "nf4"
    lora_r: int
    lora_alpha: int
    lora_dropout: float
    targets: tuple
    per_device_batch: int
    grad_accum: int
    lr: float
    epochs: float
    optim: str
    weight_decay: float = 0.0
    grad_ckpt: bool = True
    save_steps: int = 10
    save_total_limit: int = 3
    logging_steps: int = 10
    padding: str = "max_length"
    space_before_end: bool = True
    system: str = QWEN3_SYSTEM
    deepspeed: str | None = None
    output_dir: str = "./finetuned/out"
    rope_scaling: str = "keep"                # "none" = E7's rope_scaling=None override
    max_length: int = 512
    pad_to_eos: bool = True


PRESETS = {
    "qwen3-8b-lora": FinetunePreset(
        "qwen3-8b-lora", "Fine-Tuning/qwen3-8b-lora.py:114-178", "qwen3-8b", None, 16, 32, 0.05,
        ("q_proj", "k_proj", "v_proj", "o_proj"), 2, 4, 1e-4, 3, "adamw_torch", save_steps=100, save_total_limit=2,
        padding="longest", space_before_end=False, output_dir="./finetuned/qwen3-8b-lora", pad_to_eos=False),
    "qwen3-8b-lora-dist": FinetunePreset(
        "qwen3-8b-lora-dist", "Fine-Tuning/qwen3-8b-lora-dist.py:109-173", "qwen3-8b", None, 8, 16, 0.1,
        ("q_proj", "v_proj"), 2, 2, 5e-5, 3, "adamw_torch", weight_decay=0.01, save_steps=50, save_total_limit=2,
        output_dir="./finetuned/qwen3-8b-lora-dist"),
    "qwen3-8b-qlora": FinetunePreset(
        "qwen3-8b-qlora", "Fine-Tuning/qwen3-8b-qlora.py:86-140", "qwen3-8b", "nf4", 8, 16, 0.1,
        ("q_proj", "v_proj"), 4, 1, 5e-5, 3, "paged_adamw_8bit", output_dir="./finetuned/qwen3-8b-qlora"),
    "qwen3-8b-qlora-dist": FinetunePreset(
        "qwen3-8b-qlora-dist", "Fine-Tuning/qwen3-8b-qlora-dist.py:96-175", "qwen3-8b", "nf4", 8, 16, 0.1,
        ("q_proj", "v_proj"), 2, 2, 5e-5, 3, "paged_adamw_8bit", output_dir="./finetuned/qwen3-8b-qlora-dist"),
    "qwen3-14b-qlora-dist": FinetunePreset(
        "qwen3-14b-qlora-dist", "Fine-Tuning/qwen3-14b-qlora-dist.py", "qwen3-14b", "nf4", 8, 16, 0.1,
        ("q_proj", "v_proj"), 2, 2, 5e-5, 3, "paged_adamw_8bit", output_dir="./finetuned/qwen3-14b-qlora-dist"),
    "qwen3-14b-qlora-dist-deepspeed": FinetunePreset(
        "qwen3-14b-qlora-dist-deepspeed", "Fine-Tuning/qwen3-14b-qlora-dist-deepspeed.py:95-164", "qwen3-14b",
        "nf4", 8, 16, 0.1, ("q_proj", "v_proj"), 2, 2, 5e-5, 10, "paged_adamw_8bit", grad_ckpt=False,
        deepspeed="configs/ds_zero3_config.json", output_dir="./finetuned/qwen3-14b-qlora-zero3"),
    "deepseek-r1-0528-qwen3-8b-qlora-dist": FinetunePreset(
        "deepseek-r1-0528-qwen3-8b-qlora-dist", "Fine-Tuning/deepseek-r1-0528-qwen3-8b-qlora.dist.py:99-141",
        "deepseek-r1-0528-qwen3-8b", "nf4", 8, 16, 0.1, ("q_proj", "v_proj"), 2, 2, 5e-5, 5, "paged_adamw_8bit",
        space_before_end=False, system=DEEPSEEK_R1_SYSTEM, rope_scaling="none",
        output_dir="./finetuned/deepseek-r1-0528-qwen3-8b-qlora-dist"),
    "deepseek-r1-distill-1.5b-lora": FinetunePreset(
        "deepseek-r1-distill-1.5b-lora", "Scripts/fine-tuning/01-*.py:7-105", "deepseek-r1-distill-qwen-1.5b", None, 8, 16, 0.05,
        ("q_proj", "v_proj"), 4, 8, 2e-5, 3, "adamw_torch", save_steps=500, grad_ckpt=False,
        output_dir="./finetuned/deepseek-r1-distill-1.5b-lora"),
}
