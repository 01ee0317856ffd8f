"""Model zoo."""
from .common import CausalLMOutput, KVCache  # noqa: F401
from .qwen3 import (PRESETS as QWEN3_PRESETS, BitsAndBytesConfig, Qwen3Config,  # noqa: F401
                    Qwen3ForCausalLM, qwen3_config)
