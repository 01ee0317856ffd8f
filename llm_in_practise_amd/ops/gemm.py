"""Frozen-base GEMM dispatch: which kernel computes ``x · Wᵀ`` and ``dY · W``.

* Training / prefill sizes (M >= 256): the hand-written MFMA GEMM ``gemm4w`` (csrc/kernels/gemm4w*.hip) —
  forward with the residual in its epilogue, backward dX reading W as stored (transposed-B), split-K by its
  own cost model.  An NF4 base (QLoRA) either feeds its 4-bit codes straight into gemm4w (the NF4
  dequant-GEMM: the codes expanded to bf16 between the load and the LDS B image) or is expanded once per
  step at HBM speed (``nf4_dequant3_k``) when that copy serves two GEMMs (forward + dX): ``_nf4_w4``.
* Decode sizes: the split-K weight-streaming kernels (``skinny.hip``, ``gemv_w4``).
* Shapes no kernel takes (CPU tensors, K % 64): torch.
* ``GEMM_STATS`` counts every GEMM launch by form (bench.py's kernel-provenance record).

The LoRA op built on these is ``ops/linear.py``; the fused SwiGLU MLP ``ops/mlp.py``; the chunked LM-head loss
``ops/loss.py``.  Reference role: bitsandbytes' dequantize + cuBLAS (``Fine-Tuning/qwen3-8b-qlora-dist.py:102-110``).
"""
from __future__ import annotations

import collections
import os

import torch

from ..quant.nf4 import NF4Weight, dequantize_nf4
from ._native import native

_MIN_M = 256     # training / prefill-sized GEMMs: gemm4w and the fused LoRA paths

# GEMM launches by form since the last clear (bench.py provenance): "gemm4w" (bf16 B operand), "gemm4w-nf4"
# (the NF4 codes read in-kernel), "nf4-expansion" (one bf16 copy of an NF4 base), "decode" (skinny / gemv
# weight-streaming kernels), "library" (torch.matmul fallback for shapes gemm4w does not take)
GEMM_STATS: collections.Counter = collections.Counter()


def _count(form: str, n: int = 1):
    GEMM_STATS[form] += n


def _g4w_ok(a: torch.Tensor, w: torch.Tensor, bt: bool) -> bool:
    """Shapes / strides the gemm4w kernel takes for a bf16 weight: a [M, K] row-major (row stride % 8),
    w [N, K] (or [K, N] when bt) with unit inner stride, training-sized M — the same predicate the
    binding enforces (``gemm4w_supported``: K % 64, N % 8, every operand's byte extent < 4 GiB), so an
    oversized operand falls back here instead of failing in the kernel's TORCH_CHECK."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and a.dim() == 2
            and w.dim() == 2 and a.shape[0] >= _MIN_M and a.stride(1) == 1 and w.stride(1) == 1
            and a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0):
        return False
    K = a.shape[1]
    if (w.shape[0] if bt else w.shape[1]) != K:
        return False
    N = w.shape[1] if bt else w.shape[0]
    return bool(native().gemm4w_ok(a.shape[0], N, K, a.stride(0), w.stride(0), bt, False))


def _w4_ok(a: torch.Tensor, q: NF4Weight, bt: bool) -> bool:
    """An NF4 base the gemm4w kernel reads as codes (K9): forward x·deq(W)ᵀ (bt=False, a [M, K_w]) or
    dX = dY·deq(W) (bt=True, a [M, N_w]); blocksize 64, both dims multiples of 64, M > 8."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and a.dim() == 2 and a.shape[0] > 8
            and a.stride(1) == 1 and a.data_ptr() % 16 == 0 and q.kernel_ok()):
        return False
    n, k = q.shape
    if a.shape[1] != (n if bt else k):
        return False
    return bool(native().gemm4w_ok(a.shape[0], k if bt else n, a.shape[1], a.stride(0), 0, bt, True))


def _w4_gemm(a: torch.Tensor, q: NF4Weight, bt: bool, c: torch.Tensor | None = None) -> torch.Tensor:
    """gemm4w on NF4 codes: a·deq(W)ᵀ (+ c) or, bt, a·deq(W) (+ c)."""
    codes, sc = q.g4w_pack()
    n, k = q.shape
    _count("gemm4w-nf4")
    return native().gemm4w(a, codes, c, 0, bt, 0, 0, sc, k if bt else n)


def _nf4_dequant_bf16(q: NF4Weight) -> torch.Tensor:
    """One bf16 expansion of an NF4 base (HBM speed)."""
    n, k = q.shape
    _count("nf4-expansion")
    return native().nf4_dequant_fast(q.codes, q.gemv_scales(), n, k)


# Which NF4 form a call takes (LIPA_NF4_GEMM = w4 | expand | auto).  Measured per GEMM at the Qwen3-8B
# shapes (profiles/r4/gemm4w_nf4_ab.txt): the in-kernel expansion costs 1.1-1.2x the bf16 gemm4w time
# (the 3-VALU-per-element table lookup is only partly hidden beside 16x16x32 MFMAs), the same as an
# expansion + bf16 GEMM when that copy serves ONE GEMM.  "auto" therefore expands where the copy is
# reused — a training forward whose backward needs dX (the copy is kept for it: ≈14 GB transient for
# Qwen3-8B), a checkpointed layer (one expansion per optimizer step, below) — and feeds the codes
# straight in everywhere else (inference, no-grad prefill, frozen inputs): no transient bf16 weights.
# "w4" everywhere is the memory-lean training mode (peak HBM ≈ the 4-bit model + activations).
_NF4_MODE = os.environ.get("LIPA_NF4_GEMM", "auto")


def _nf4_w4(reused: bool) -> bool:
    if _NF4_MODE == "w4":
        return True
    if _NF4_MODE == "expand":
        return False
    return not (reused or _IN_CKPT[0])


# NF4-aware activation checkpointing: inside a checkpointed layer (its forward AND its backward
# recompute) the bf16 expansion of each frozen NF4 base is made once per optimizer step and reused —
# the reference-faithful step (gradient checkpointing + sequential GA micro-steps) otherwise expands
# every weight 2 × GA times per step.  The copies are held in ONE registry, bounded by
# LIPA_CKPT_NF4_CACHE_GB (default 32; 0 = off: every call expands), and released eagerly when the
# optimizer steps (``nf4_cache_advance``: optim/adamw.py, parallel/zero.py; an optimizer that never
# calls it keeps at most the budget).  Memory: the budget is the cost — Qwen3-8B's bases expand to
# 13.9 GB (peak HBM of the faithful bench step: README §3).
_CKPT_BUDGET = float(os.environ.get("LIPA_CKPT_NF4_CACHE_GB", "32")) * 2 ** 30
_IN_CKPT = [0]
_CACHE: dict = {}        # id(NF4Weight) -> (weight, bf16 expansion)
_CACHE_BYTES = [0]


def nf4_cache_advance():
    """Called by the optimizers at every step: the expanded copies of the finished step are released."""
    _CACHE.clear()
    _CACHE_BYTES[0] = 0


def _nf4_expand(q: NF4Weight) -> torch.Tensor:
    """The bf16 expansion for the "expand" form (cached inside checkpointed layers, see above)."""
    if _IN_CKPT[0]:
        hit = _CACHE.get(id(q))
        if hit is not None and hit[0] is q:
            return hit[1]
    w = _nf4_dequant_bf16(q)
    if _IN_CKPT[0] and _CACHE_BYTES[0] + w.numel() * 2 <= _CKPT_BUDGET:
        _CACHE[id(q)] = (q, w)
        _CACHE_BYTES[0] += w.numel() * 2
    return w


def head_logits(h: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """LM-head logits of serving rows, batch-invariant: on the GPU always gemm4w with one K-split — every logit
    is one lane's fp32 accumulation over K in the same order whatever the tile shape the planner picks for this
    row count — so a request's greedy tokens do not depend on how many rows share the call (continuous batching,
    hipGraph buckets, the pipelined engine).  A library GEMM's algorithm (and rounding) changes with M.  The
    head is weight-streaming at decode sizes (151936 × 4096 bf16 = 1.2 GB per call): the kernel reads each
    weight panel once, as a GEMV would."""
    x = h.reshape(-1, h.shape[-1])
    if not x.is_contiguous():
        x = x.contiguous()
    if (x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and weight.dim() == 2
            and weight.stride(1) == 1 and x.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0
            and weight.shape[1] == x.shape[1]
            and native().gemm4w_ok(x.shape[0], weight.shape[0], x.shape[1], x.stride(0), weight.stride(0), False,
                                   False)):
        _count("gemm4w")
        y = native().gemm4w(x, weight, None, 1, False)
    else:
        y = _base_gemm(x, weight)
    return y.view(*h.shape[:-1], weight.shape[0])


def _base_gemm(x, base, ext_a=None, ext_b=None, residual=None):
    if isinstance(base, NF4Weight):
        if x.shape[0] <= 8 and base.kernel_ok():   # decode: weight-streaming GEMV, no MFMA tile
            n, k = base.shape
            _count("decode")
            y = native().gemv_w4(x, base.codes, base.gemv_scales(), None, n, base.blocksize,
                                 residual if ext_a is None else None)
            if ext_a is not None:
                y = y + ext_a @ ext_b.t()
                if residual is not None:
                    y = y + residual
            return y
        if _w4_ok(x, base, False):                  # the NF4 dequant-GEMM (gemm4w reads the codes)
            y = _w4_gemm(x, base, False, None if residual is None else residual.contiguous())
            return y if ext_a is None else y.addmm_(ext_a, ext_b.t())
        w = _nf4_dequant_bf16(base) if (base.kernel_ok() and x.is_cuda) else dequantize_nf4(base, x.dtype)
        return _base_gemm(x, w, ext_a, ext_b, residual)
    M, K = x.shape
    N = base.shape[0]
    if (x.is_cuda and M <= 16 and N <= 8192 and K <= 8192 and N % 16 == 0 and K % 64 == 0 and x.stride(0) % 8 == 0
            and x.stride(1) == 1 and base.is_contiguous()):
        # decode-sized q|k|v / o projections: the split-K weight-streaming MFMA kernel
        # (csrc/kernels/skinny.hip) beats hipBLASLt's latency-bound 23 µs by 25-45 % and fuses
        # the residual; the wide gate|up / long-K down stay on hipBLASLt (≥ 5 TB/s there)
        _count("decode")
        y = native().gemm_skinny(x, base, residual)
        return y if ext_a is None else y.addmm_(ext_a, ext_b.t())
    if _g4w_ok(x, base, False):
        _count("gemm4w")
        y = native().gemm4w(x, base, None if residual is None else residual.contiguous(), 0, False)
        return y if ext_a is None else y.addmm_(ext_a, ext_b.t())
    # shapes gemm4w does not take (CPU, M < 256, K % 64): torch — residual = addmm's beta term, the LoRA
    # K-slice one rank-Σr update
    _count("library")
    y = torch.addmm(residual, x, base.t()) if residual is not None else x @ base.t()
    if ext_a is not None:
        y.addmm_(ext_a, ext_b.t())
    return y


def _dense_dx(dy: torch.Tensor, w: torch.Tensor, c: torch.Tensor | None = None) -> torch.Tensor:
    """dX = dY·W (+ c) for a bf16 [N, K] weight: gemm4w's transposed-B form (W read as stored; split-K when
    the output has fewer tiles than CUs, e.g. gate|up dX at M = 2048), else torch."""
    if _g4w_ok(dy, w, True):
        _count("gemm4w")
        return native().gemm4w(dy, w, c, 0, True)
    _count("library")
    return dy @ w if c is None else torch.addmm(c, dy, w)


def _base_gemm_t(dy, base, ext_a=None, ext_b=None, c=None):
    """dX = dY·W (+ c) (+ ext_a · ext_bᵀ, ext_b given as [K, R])."""
    if isinstance(base, NF4Weight):
        if _w4_ok(dy, base, True):
            dx = _w4_gemm(dy, base, True, c)
            return dx if ext_a is None else dx.addmm_(ext_a, ext_b.t())
        base = _nf4_dequant_bf16(base) if (base.kernel_ok() and dy.is_cuda) else dequantize_nf4(base, dy.dtype)
    dx = _dense_dx(dy, base, c)
    return dx if ext_a is None else dx.addmm_(ext_a, ext_b.t())
