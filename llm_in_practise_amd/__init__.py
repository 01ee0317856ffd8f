"""llm_in_practise_amd — an MI355X-native (gfx950 / CDNA4) LLM training, fine-tuning,
quantisation and serving stack with the capabilities of iKubernetes/llm-in-practise.

Layers:
  runtime/   device + torchrun env contract (L0)
  parallel/  RCCL/gloo process groups, DDP, ZeRO-1/2/3(+offload), ds_config semantics (L1/L3)
  ops/       autograd ops; HIP kernels on gfx950, pure-PyTorch references on CPU (L2)
  models/    MiniGPT, GPTLike, DeepSeekLike (MLA+MoE), Qwen3 / DeepSeek-R1-Qwen3 (L4)
  peft/ quant/  LoRA / QLoRA (NF4) / GPTQ / AWQ (L5)
  optim/ train/ training loop, HF-Trainer-compatible arguments, checkpoints (L6)
  cli/       entry points mirroring the reference scripts (L7)
  infer/     KV-cache generation, sampling, OpenAI-compatible server, moderation (L8)
"""

__version__ = "0.2.0"

import os as _os

# RCCL / CUDA-tensor IPC on this ROCm image only works through dmabuf: the legacy IPC path must be
# off BEFORE the first HIP call of the process (HIP reads it at runtime init), so it is set at
# package import rather than next to init_process_group.
_os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from .runtime.device import get_device, is_gfx950  # noqa: F401
