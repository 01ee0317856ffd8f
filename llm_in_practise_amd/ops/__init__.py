"""Op layer: HIP kernels for gfx950 on GPU tensors, PyTorch references on CPU."""
from .activation import gelu, swiglu_fused  # noqa: F401
from .attention import flash_attention, sdpa_bshd  # noqa: F401
from .embedding import Embedding, embedding  # noqa: F401
from .linear import LoraBranch, fused_linear  # noqa: F401
from .loss import cross_entropy, fused_linear_cross_entropy, shift_labels  # noqa: F401
from .norm import LayerNorm, RMSNorm, layer_norm, rms_norm  # noqa: F401
from .rope import apply_rope, qk_norm_rope  # noqa: F401
from ._native import has_native, native  # noqa: F401
