"""Quantisation (Track F): NF4 (QLoRA), int4 W4A16 (GPTQ / AWQ)."""
from .nf4 import NF4Weight, concat_nf4, dequantize_nf4, quantize_nf4  # noqa: F401
