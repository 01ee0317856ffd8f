"""PEFT-compatible LoRA / QLoRA without the peft package."""
from .lora import (Linear4bit, LoraConfig, LoraLayer, PeftModel, TaskType, get_peft_model,  # noqa: F401
                   prepare_model_for_kbit_training, quantize_model_nf4)
