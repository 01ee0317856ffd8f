"""Frozen-base linear with LoRA branches (K8) over NF4 or bf16 bases (K9).

One op covers every projection of the stack:

    y[:, c0:c1] (+)= x · deq(W)ᵀ  +  Σ_i s_i · (drop_i(x) · A_iᵀ) · B_iᵀ   (+ residual)

* ``base`` is a bf16 ``[N, K]`` tensor (LoRA / full fine-tune) or an :class:`NF4Weight`
  (QLoRA).  Several projections that share an input (q|k|v, gate|up) are row-concatenated
  into one base and one GEMM; each LoRA branch owns a column range ``[c0, c1)``.
* Every frozen-base GEMM at training / prefill sizes is the hand-written MFMA kernel ``gemm4w``
  (csrc/kernels/gemm4w.hip) — there is no library GEMM on the path: forward x·Wᵀ with the residual in
  its epilogue, backward dY·W reading W as stored (the transposed-B form), split-K by its own cost model.
  - An NF4 base (K9) takes one of two forms, chosen per call (``_nf4_w4``): the NF4 dequant-GEMM —
    gemm4w reads the 4-bit codes (``NF4Weight.g4w_pack``) and expands each quant block to bf16 between
    the load and its LDS B image, no bf16 copy of the base anywhere — or one HBM-speed expansion
    (``nf4_dequant3_k``) whose bf16 copy serves the forward AND the dX GEMM.
  - The LoRA branches ride inside gemm4w where their shapes allow: the adapters' B term as extra MFMA
    K-steps of the forward (``gemm4w_lora``), the dropout-masked input-gradient term in the dX GEMM's
    prologue (``gemm4w_loradx``); the rank-r projections, dB and dA run in ``lora.hip`` (``lora_proj2`` /
    ``lora_proj_m`` forward, ``lora_proj_pair`` / ``lora_acc_quad`` / ``lora_acc_jobs`` backward).
    Other shapes fall back to ``lora_apply`` (B term added into the adapters' column blocks) and
    ``lora_acc`` / ``lora_dx2``.
  - Decode sizes (M ≤ 16) use the split-K weight-streaming kernels (``skinny.hip``, ``gemv_w4``).
  - Shapes gemm4w does not take (K % 64 ≠ 0, tiny M, CPU tensors) run ``torch.matmul``.
* The SwiGLU MLP block bypasses this op when it carries no adapters (``ops/mlp.py``).
* ``GEMM_STATS`` counts every GEMM launch by form (the bench record's provenance).

Reference parity: PEFT ``LoraConfig(r, lora_alpha, lora_dropout, target_modules)``
(``Fine-Tuning/qwen3-8b-qlora.py:107-114``), scaling = alpha / r.
"""
from __future__ import annotations

import collections
import dataclasses
import os

import torch
import torch.nn.functional as F

from ..quant.nf4 import NF4Weight, dequantize_nf4
from ._native import native, use_native

EXT_ALIGN = 32   # the kernels consume the LoRA K-slice in MFMA K-steps of 32
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


# LoRA kernel forms (the A/B-measured winners of round 2, fixed; profiles/lora_acc_mfma_ab.txt):
# q_proj + v_proj with dropout — the forward's lora_proj2 stores the keep bits (1 bit per element and
# branch) for the backward instead of re-hashing; two-branch backward launches (lora_proj_pair /
# lora_acc_pair); the LoRA dX term as the dX GEMM's C matrix + a separate dA launch
_KEEP_BITS = True
_PAIR_BWD = True
_DX_C = True


@dataclasses.dataclass
class LoraBranch:
    a: torch.Tensor          # [r, K]
    b: torch.Tensor          # [n, r]
    scaling: float
    dropout: float
    c0: int
    c1: int


def _pad_cols(t: torch.Tensor, mult: int = EXT_ALIGN) -> torch.Tensor:
    r = t.shape[-1]
    rp = (r + mult - 1) // mult * mult
    if rp == r:
        return t.contiguous()
    return F.pad(t, (0, rp - r)).contiguous()


def head_logits(h: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """LM-head logits of serving rows through the same dispatch as the projections: decode-sized row counts take
    the split-K weight-streaming kernel, whose per-row result does not depend on how many rows share the call
    (the library GEMM's algorithm — and rounding — changes with M), so a request's greedy tokens do not depend on
    the batch it was decoded in (continuous batching, hipGraph buckets, the pipelined engine)."""
    x = h.reshape(-1, h.shape[-1])
    if not x.is_contiguous():
        x = x.contiguous()
    return _base_gemm(x, weight).view(*h.shape[:-1], weight.shape[0])


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


_KEY = [0x5DEECE66D << 20]

# "gradient final" listeners (parallel/ddp.py bucket overlap): called with the parameter whose
# flat-buffer gradient a fused backward kernel has just accumulated in place (those gradients
# bypass autograd's AccumulateGrad, so post_accumulate_grad_hooks do not fire for them)
_GRAD_READY: list = []


def register_grad_ready(fn):
    import weakref
    ref = weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda f=fn: f)
    _GRAD_READY.append(ref)
    return ref


def _notify_grad_ready(p):
    dead = False
    for r in _GRAD_READY:
        f = r()
        if f is None:
            dead = True
        else:
            f(p)
    if dead:
        _GRAD_READY[:] = [r for r in _GRAD_READY if r() is not None]


def next_dropout_key() -> int:
    """Counter-based dropout stream: every call gets a fresh 63-bit key (deterministic given
    the seed set by :func:`seed_dropout`)."""
    _KEY[0] = (_KEY[0] + 0x9E3779B97F4A7C15) & 0x7FFFFFFFFFFFFFFF
    return _KEY[0]


def seed_dropout(seed: int):
    _KEY[0] = (int(seed) * 0x2545F4914F6CDD1D) & 0x7FFFFFFFFFFFFFFF


_CKPT_REENTRANT = os.environ.get("LIPA_CKPT_REENTRANT", "1") == "1"
# HF semantics by default (the whole layer recomputed); "selective" keeps every GEMM output of the
# first forward (~78 MB per Qwen3-8B layer per 1024 tokens) and is opt-in
_CKPT_POLICY = os.environ.get("LIPA_CKPT_POLICY", "full")


def checkpoint(fn, *args, use_reentrant: bool | None = None, policy: str | None = None):
    """Activation checkpointing of one layer that replays the SAME LoRA dropout masks.

    ``use_reentrant`` selects torch's form (HF's ``gradient_checkpointing_kwargs={"use_reentrant": …}``,
    ``Fine-Tuning/qwen3-8b-qlora-dist.py:162-163``; default: LIPA_CKPT_REENTRANT, on).  ``policy``:
    ``"full"`` (default, LIPA_CKPT_POLICY) recomputes the whole layer in backward (HF's behaviour);
    ``"selective"`` records the GEMM outputs in the first forward and replays them in the recompute —
    only RMSNorm, q/k-norm + RoPE and attention run again (the stash below): faster, but it holds
    ≈ 78 MB per Qwen3-8B layer per 1024 tokens from the forward until the backward.

    The fused LoRA kernels draw their dropout mask from the host key stream above, not from
    torch's RNG, so torch's ``preserve_rng_state`` does not cover them: a plain
    ``torch.utils.checkpoint`` recompute would draw fresh keys and the backward would differentiate
    a different mask than the forward applied.  Here the key-stream position at the first (forward)
    call is remembered and restored for the recompute, then the live stream is put back — the
    masks match exactly and the stream advances once per real forward.  Reference:
    ``Fine-Tuning/qwen3-8b-lora.py:123`` (gradient checkpointing + ``lora_dropout``).  The reentrant
    form's first forward builds no graph (no saved-tensor pack hooks: ~2k per step at Qwen3-8B, the
    host-side cost of the checkpointed step, profiles/baseline_configs_r2_end.txt)."""
    import torch.utils.checkpoint as ckpt
    reentrant = _CKPT_REENTRANT if use_reentrant is None else bool(use_reentrant)
    policy = policy or _CKPT_POLICY
    if policy not in ("full", "selective"):
        raise ValueError(f"checkpoint policy {policy!r}: 'full' or 'selective'")
    stash = _Stash() if policy == "selective" else None
    state: list = []

    def run(*a):
        _IN_CKPT[0] += 1
        prev = list(_SAC)
        try:
            if not state:                      # the forward pass
                state.append(_KEY[0])
                if stash is not None:
                    _SAC[:] = ["record", stash]
                return fn(*a)
            live = _KEY[0]                     # the recompute inside backward
            _KEY[0] = state[0]
            if stash is not None:
                stash.pos = 0
                _SAC[:] = ["replay", stash]
            try:
                return fn(*a)
            finally:
                _KEY[0] = live
        finally:
            _SAC[:] = prev
            _IN_CKPT[0] -= 1

    if reentrant:
        # the first forward runs without building a graph; it needs an input that requires grad for the
        # recompute to reach the LoRA parameters (layer 0's input is the frozen embedding) — the role of
        # HF's enable_input_require_grads()
        args = tuple(a.detach().requires_grad_() if isinstance(a, torch.Tensor) and i == 0 and
                     a.is_floating_point() and not a.requires_grad else a for i, a in enumerate(args))
        return ckpt.checkpoint(run, *args, use_reentrant=True)
    return ckpt.checkpoint(run, *args, use_reentrant=False)


def bf16_view(p: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """The optimizer-maintained low-precision shadow of a fp32 trainable parameter
    (written by the fused AdamW kernel every step), else a cast."""
    sh = getattr(p, "_lipa_shadow", None)
    if sh is not None and sh.dtype == dtype:
        return sh
    return p.detach().to(dtype)


def deterministic() -> bool:
    """Bit-reproducible LoRA gradients (``LIPA_DETERMINISTIC=1`` or
    ``torch.use_deterministic_algorithms(True)``): fixed-order partial sums instead of fp32
    atomics in the fused LoRA backward (≈0.5 % slower)."""
    import os
    return os.environ.get("LIPA_DETERMINISTIC", "0") == "1" or torch.are_deterministic_algorithms_enabled()


_ZBUF: dict = {}


def _zero_buffer(tag: str, rows: int, cols: int, like: torch.Tensor) -> torch.Tensor:
    """A persistent zero-initialised scratch tensor.  The LoRA extra K-slice buffers only ever
    get the same block regions rewritten (B blocks / the x·Aᵀ columns); everything else must
    stay zero, so one allocation + fill serves every step instead of a fill kernel per call.
    Consumers are stream-ordered (each buffer is read by the GEMM launched right after it is
    written), so sharing a buffer between projections of the same shape is safe."""
    key = (tag, rows, cols, like.dtype, like.device)
    t = _ZBUF.get(key)
    if t is None:
        t = torch.zeros(rows, cols, dtype=like.dtype, device=like.device)
        _ZBUF[key] = t
    return t


def _lora_epi_ok(x, base, wdq, weight, branches) -> bool:
    """The branches fit the gemm4w LoRA epilogue: ranks multiples of 8 (≤ 128 in all), training-sized M, the
    base GEMM itself on gemm4w (a bf16 weight / expansion, or NF4 codes)."""
    if not (x.shape[0] >= _MIN_M and all(br.a.shape[0] % 8 == 0 for br in branches)
            and sum(br.a.shape[0] for br in branches) <= 128):
        return False
    if wdq is not None:
        return _g4w_ok(x, wdq, False)
    if isinstance(base, NF4Weight):
        return _w4_ok(x, base, False)
    return weight is not None and not weight.requires_grad and _g4w_ok(x, weight, False)


# the two-branch (q_proj + v_proj) and multi-adapter kernel families; the GPU tests switch these off to
# check them against the per-adapter kernels, which stay the general path for every other shape
_PAIR = True
_MULTI = True


def _pair_ok(x, branches) -> bool:
    """Two rank-<=8 adapters on one fused projection (q_proj + v_proj): the two-branch kernels."""
    return _PAIR and len(branches) == 2 and x.is_cuda and all(br.a.shape[0] <= 8 for br in branches)


def _multi_ok(x, branches) -> bool:
    """1-4 adapters of rank 8 or 16 on one projection that are not the rank-8 q+v pair (BASELINE #2: q, k, v
    on q|k|v, o alone): the multi-adapter kernels — one pass over x for every branch's s·D(x)·Aᵀ with the
    keep bits stored (``lora_proj_m``), every g_b in one launch (``lora_proj_cols``), every dB and dA in
    one launch (``lora_acc_jobs``), the masked dX term inside the dX GEMM (1-2 branches: gemm4w_loradx)
    or as its C matrix (``lora_dxc``).  Training-sized M only; decode keeps the per-branch kernels.
    Reference config: ``Fine-Tuning/qwen3-8b-lora.py:128-141`` (r 16 / alpha 32 / dropout 0.05 on q, k, v, o)."""
    return (_MULTI and x.is_cuda and 1 <= len(branches) <= 4 and x.shape[0] >= _MIN_M
            and not _pair_ok(x, branches)
            and all(br.a.shape[0] in (8, 16) and (br.c1 - br.c0) % 512 == 0 for br in branches))


def _fast_lora_ok(x, branches) -> bool:
    """Shapes the fused LoRA branch kernels (csrc/kernels/lora.hip) take."""
    K = x.shape[1]
    return (K % 128 == 0 and all(br.a.shape[0] <= 16 and (br.c1 - br.c0) % 128 == 0 for br in branches))


# Selective activation checkpointing (``checkpoint(..., policy="selective")``): the checkpointed
# layer's first forward RECORDS the outputs of its GEMM ops (the frozen-base projections with their LoRA
# side products, the fused SwiGLU MLP) in a per-call stash; the recompute inside backward REPLAYS them
# instead of launching the GEMMs again, and recomputes only the cheap ops between them (RMSNorm, q/k-norm
# + RoPE, attention).  The stash holds ≈ 78 MB per Qwen3-8B layer at 1024 tokens (y_qkv, y_o, gu, y_down
# + the rank-r LoRA projections) until the backward consumes it.
_SAC: list = [None, None]      # (mode "record" | "replay", stash list)


def _sac_recording() -> bool:
    return _SAC[0] == "record"


def sac_put(item):
    if _SAC[0] == "record":
        _SAC[1].append(item)


def sac_take():
    """The next recorded op output when replaying, else None."""
    if _SAC[0] != "replay":
        return None
    st = _SAC[1]
    i = st.pos
    st.pos += 1
    item, st[i] = st[i], None
    return item


class _Stash(list):
    pos = 0


class _FusedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, meta, *ab):
        base, branches, training = meta
        dense = not isinstance(base, NF4Weight)
        replay = sac_take()
        if replay is not None:   # selective checkpointing: this op's outputs from the layer's first forward
            y, xa_list, keys, ctx.masks, ctx.bts, expanded = replay
            for k in keys:       # the key stream advances exactly as in the recorded forward
                if k is not None:
                    next_dropout_key()
            fast = bool(branches) and _fast_lora_ok(x, branches)
            wdq = _nf4_expand(base) if expanded else None
            return _FusedLinearFn._finish(ctx, x, residual, weight, meta, ab, y, xa_list, keys, fast, wdq)
        xa_list, keys = [], []
        ext_a = ext_b = None
        ctx.masks = None
        fast = bool(branches) and _fast_lora_ok(x, branches)
        # (grad mode is off inside forward: ask autograd; a recording first forward keeps the LoRA side
        # products too — the replay's backward needs them)
        need_xa = any(ctx.needs_input_grad[5:]) or _sac_recording()
        # "apply" form: the adapters' B term inside gemm4w (epi) or added by lora_apply into ONLY their column
        # blocks of the base GEMM's output (no K-slice buffers, no per-call B copies, no rank-Σr update over
        # all N columns); the K-slice form below serves the CPU / odd-shaped rest
        apply = fast and x.is_cuda and len(branches) <= 4
        wdq = None
        if not dense and x.shape[0] > 8 and base.kernel_ok() and x.is_cuda and not _nf4_w4(ctx.needs_input_grad[0]):
            wdq = _nf4_expand(base)     # the expand form: this copy also serves the dX GEMM
        # the adapters' B term as extra MFMA K-steps of the base GEMM (gemm4w LoRA epilogue): xa in bf16
        # slots of a 32·k-wide buffer, no lora_apply pass over y
        epi = apply and _lora_epi_ok(x, base, wdq, weight, branches)
        xa32 = None
        if epi:
            kofs, k = [], 0
            for br in branches:
                kofs.append(k)
                k += br.a.shape[0]
            xa32 = _zero_buffer(f"lora_xa32_{(k + 31) // 32}", x.shape[0], (k + 31) // 32 * 32, x)
        if apply:
            pair = _pair_ok(x, branches)
            if pair:
                ps = [br.dropout if training else 0.0 for br in branches]
                keys = [next_dropout_key() if p > 0 else None for p in ps]
                a0, a1 = bf16_view(ab[0], x.dtype), bf16_view(ab[2], x.dtype)
                # training with dropout on both: keep the masks' bits (2 bits / element of x) for lora_acc2
                masks = (torch.empty(2, x.shape[0], x.shape[1] // 8, dtype=torch.uint8, device=x.device)
                         if need_xa and all(k is not None for k in keys) and _KEEP_BITS else None)
                xa2 = native().lora_proj2(x, a0, a1, None if xa32 is None else xa32[:, :a0.shape[0] + a1.shape[0]], True,
                                          ps[0], keys[0] or 0, branches[0].scaling, ps[1], keys[1] or 0,
                                          branches[1].scaling, masks)
                ctx.masks = masks
                r0 = a0.shape[0]
                xa_list = [xa2[:, :r0], xa2[:, r0:]]
            elif _multi_ok(x, branches):
                ps = [br.dropout if training else 0.0 for br in branches]
                keys = [next_dropout_key() if p > 0 else None for p in ps]
                # every branch's keep bits (an all-ones plane for a branch without dropout) for the backward
                masks = (torch.empty(len(branches), x.shape[0], x.shape[1] // 8, dtype=torch.uint8, device=x.device)
                         if need_xa and any(k is not None for k in keys) else None)
                obs = [None if xa32 is None else xa32[:, kofs[i]:kofs[i] + br.a.shape[0]]
                       for i, br in enumerate(branches)]
                xa_list = list(native().lora_proj_m(x, [bf16_view(a, x.dtype) for a in ab[0::2]], obs, True, ps,
                                                    [k or 0 for k in keys], [br.scaling for br in branches], masks))
                ctx.masks = masks
            else:
                for bi, (br, a) in enumerate(zip(branches, ab[0::2])):
                    p = br.dropout if training else 0.0
                    key = next_dropout_key() if p > 0 else None
                    ob = None if xa32 is None else xa32[:, kofs[bi]:kofs[bi] + a.shape[0]]
                    xa_list.append(native().lora_proj(x, 0, x.shape[1], bf16_view(a, x.dtype), ob, True, p,
                                                      key or 0, br.scaling))
                    keys.append(key)
        elif branches:
            N = base.shape[0]
            rtot = sum(br.a.shape[0] for br in branches)
            rp = (rtot + EXT_ALIGN - 1) // EXT_ALIGN * EXT_ALIGN
            layout = tuple((br.c0, br.c1, br.a.shape[0]) for br in branches)
            if x.is_cuda and not torch.cuda.is_current_stream_capturing():
                ext_b = _zero_buffer(f"lora_b{layout}", N, rp, x)
                ext_a = _zero_buffer(f"lora_xa{rtot}", x.shape[0], rp, x) if fast else None
            else:
                ext_b = x.new_zeros(N, rp)
                ext_a = x.new_zeros(x.shape[0], rp) if fast else None
            cols, r0 = [], 0
            pair = fast and _pair_ok(x, branches)
            if pair:   # q_proj + v_proj: ONE pass over x for both adapters (lora_proj2)
                ps = [br.dropout if training else 0.0 for br in branches]
                pair_keys = [next_dropout_key() if p > 0 else None for p in ps]
                a0, a1 = bf16_view(ab[0], x.dtype), bf16_view(ab[2], x.dtype)
                rr = a0.shape[0] + a1.shape[0]
                xa2 = native().lora_proj2(x, a0, a1, ext_a[:, :rr], need_xa, ps[0], pair_keys[0] or 0,
                                          branches[0].scaling, ps[1], pair_keys[1] or 0, branches[1].scaling, None)
            for bi, (br, (a, b)) in enumerate(zip(branches, zip(ab[0::2], ab[1::2]))):
                r = a.shape[0]
                p = br.dropout if training else 0.0
                if pair:
                    key = pair_keys[bi]
                    xa = xa2[:, r0:r0 + r] if need_xa else None
                    ext_b[br.c0:br.c1, r0:r0 + r] = bf16_view(b, x.dtype)
                    xa_list.append(xa)
                    keys.append(key)
                    r0 += r
                    continue
                key = next_dropout_key() if p > 0 else None
                if fast:   # one MFMA pass: s·D(x)·Aᵀ into the ext slice (bf16) + fp32 copy for dB
                    xa = native().lora_proj(x, 0, x.shape[1], bf16_view(a, x.dtype), ext_a[:, r0:r0 + r],
                                            need_xa, p, key or 0, br.scaling)
                else:
                    xd = native().dropout_fwd(x, p, key) if key is not None else x
                    xa = xd @ bf16_view(a, x.dtype).t()                # [T, r]
                    cols.append(xa * br.scaling)
                ext_b[br.c0:br.c1, r0:r0 + r] = bf16_view(b, x.dtype)
                xa_list.append(xa)
                keys.append(key)
                r0 += r
            if not fast:
                ext_a = _pad_cols(torch.cat(cols, 1))
        ctx.bts = None
        if epi:
            bs = [bf16_view(b, x.dtype) for b in ab[1::2]]
            bts = [torch.empty(b.shape[1], b.shape[0], dtype=x.dtype, device=x.device) for b in bs] if need_xa else []
            w_op = wdq if wdq is not None else (weight if dense else None)
            res = None if residual is None else residual.contiguous()
            _count("gemm4w" if w_op is not None else "gemm4w-nf4")
            if w_op is not None:
                y = native().gemm4w_lora(x, w_op, None, 0, res, xa32, bs, [br.c0 for br in branches], kofs,
                                         bts or [None] * len(bs))
            else:
                codes, sc = base.g4w_pack()
                y = native().gemm4w_lora(x, codes, sc, base.shape[0], res, xa32, bs, [br.c0 for br in branches], kofs,
                                         bts or [None] * len(bs))
            ctx.bts = bts or None
            if not need_xa:
                xa_list = [None] * len(xa_list)
        else:
            y = _base_gemm(x, wdq if wdq is not None else (base if not dense else weight), ext_a, ext_b, residual)
        if apply and not epi:
            bs = [bf16_view(b, x.dtype) for b in ab[1::2]]
            # training: the same pass writes Bᵀ [r, n] for the backward's dy·B projection (no transpose kernel)
            bts = [torch.empty(b.shape[1], b.shape[0], dtype=x.dtype, device=x.device) for b in bs] if need_xa else []
            native().lora_apply(y, xa_list, bs, [br.c0 for br in branches], bts)
            ctx.bts = bts or None
            if not need_xa:
                xa_list = [None] * len(xa_list)
        if bias is not None:
            y = y + bias
        sac_put((y, list(xa_list), keys, ctx.masks, ctx.bts, wdq is not None))
        return _FusedLinearFn._finish(ctx, x, residual, weight, meta, ab, y, xa_list, keys, fast, wdq)

    @staticmethod
    def _finish(ctx, x, residual, weight, meta, ab, y, xa_list, keys, fast, wdq):
        branches = meta[1]
        ctx.wdq = wdq if ctx.needs_input_grad[0] else None
        ctx.meta = meta
        ctx.keys = keys
        ctx.fast = fast
        ctx.pair = bool(branches) and fast and _pair_ok(x, branches)
        # (the forward's condition for lora_proj_m: "apply" form and the multi-adapter shapes)
        ctx.multi = bool(branches) and fast and x.is_cuda and len(branches) <= 4 and _multi_ok(x, branches)
        ctx.ab_refs = ab          # the parameters themselves: fused kernels accumulate into their .grad
        ctx.has_residual = residual is not None
        # the LoRA parameters travel as ctx.ab_refs, not through save_for_backward: under non-reentrant
        # checkpointing every saved tensor costs a Python pack / unpack hook (host time of the
        # reference-faithful step), and parameters need no saving
        ctx.save_for_backward(x, weight, *[t for t in xa_list if t is not None])
        ctx.nb = len(branches)
        return y

    @staticmethod
    def backward(ctx, dy):
        base, branches, training = ctx.meta
        saved = ctx.saved_tensors
        x, weight = saved[0], saved[1]
        nb = ctx.nb
        ab = ctx.ab_refs
        xa_list = saved[2:2 + nb]
        dense = not isinstance(base, NF4Weight)
        dy = dy.contiguous()
        fast = ctx.fast
        grads_ab = [None] * (2 * nb)
        g_list = []
        done_quad = None      # ((dA_0, ret), (dA_1, ret)) when lora_acc_quad already produced both dA

        def dest(i):   # the optimizer-owned fp32 grad view (accumulate in place) or a fresh buffer
            prm = ctx.ab_refs[i]
            gr = prm.grad
            if gr is not None and getattr(prm, "_lipa_flat_grad", False) and gr.dtype == torch.float32:
                return gr, False
            return torch.zeros(prm.shape, dtype=torch.float32, device=dy.device), True

        if (ctx.multi and not deterministic() and ctx.bts is not None and all(t is not None for t in xa_list)
                and (ctx.masks is not None or all(k is None for k in ctx.keys))):
            return _multi_backward(ctx, dy, x, weight, xa_list, base, branches, dense, dest)
        # q_proj + v_proj: both adapters' s·dy_i·B_i in one launch, both dB_i in another
        pair_g = (fast and nb == 2 and ctx.bts is not None and ctx.bts[0].shape[0] == ctx.bts[1].shape[0]
                  and all(bt.shape[1] % 512 == 0 for bt in ctx.bts) and _PAIR_BWD)
        if pair_g:
            g_list = list(native().lora_proj_pair(dy, branches[0].c0, ctx.bts[0], branches[0].scaling,
                                                  branches[1].c0, ctx.bts[1], branches[1].scaling))
            xs = xa_list
            if (ctx.needs_input_grad[6] and ctx.needs_input_grad[8] and not deterministic() and xs[0] is not None
                    and xs[1] is not None and xs[0].stride(0) == xs[1].stride(0) and xs[0].shape[1] <= 8
                    and all((br.c1 - br.c0) % 128 == 0 for br in branches)):
                (o0, ret0), (o1, ret1) = dest(1), dest(3)
                # with the dropout pair's dA due too (the keep-bit path below), both dB and both dA in ONE launch
                quad = (_DX_C and ctx.pair and all(k is not None for k in ctx.keys) and ctx.masks is not None
                        and ctx.needs_input_grad[0] and ctx.needs_input_grad[5] and ctx.needs_input_grad[7]
                        and dy.shape[0] >= _MIN_M and x.shape[1] % 128 == 0
                        and g_list[0].shape[1] == xs[0].shape[1])
                if quad:
                    (a0o, aret0), (a1o, aret1) = dest(0), dest(2)
                    native().lora_acc_quad(xs[0], xs[1], dy, branches[0].c0, o0, branches[1].c0, o1, g_list[0],
                                           g_list[1], x, a0o, a1o, ctx.masks, branches[0].dropout, branches[1].dropout)
                    done_quad = ((a0o, aret0), (a1o, aret1))
                else:
                    native().lora_acc_pair(xs[0], xs[1], dy, branches[0].c0, o0, branches[1].c0, o1)
                for i, (o, ret) in ((0, (o0, ret0)), (1, (o1, ret1))):
                    if ret:
                        grads_ab[2 * i + 1] = o.to(ab[2 * i + 1].dtype)
                    else:
                        _notify_grad_ready(ctx.ab_refs[2 * i + 1])
            else:
                for i, br in enumerate(branches):
                    if ctx.needs_input_grad[5 + 2 * i + 1]:
                        out, ret = dest(2 * i + 1)
                        native().lora_acc(xa_list[i], dy, br.c0, br.c1 - br.c0, out, True, None, None, 0.0, 0,
                                          deterministic())
                        grads_ab[2 * i + 1] = out.to(ab[2 * i + 1].dtype) if ret else None
                        if not ret:
                            _notify_grad_ready(ctx.ab_refs[2 * i + 1])
        for i, br in enumerate(branches if not pair_g else ()):
            a, b = ab[2 * i], ab[2 * i + 1]
            n_i = br.c1 - br.c0
            if fast:
                bt = ctx.bts[i] if ctx.bts is not None else bf16_view(b, dy.dtype).t().contiguous()   # [r, n_i]
                g = native().lora_proj(dy, br.c0, n_i, bt, None, True, 0.0, 0, br.scaling)   # s·dy_i·B, fp32
                if ctx.needs_input_grad[5 + 2 * i + 1]:
                    out, ret = dest(2 * i + 1)                                     # dB [n_i, r] += dy_iᵀ·xa_s
                    native().lora_acc(xa_list[i], dy, br.c0, n_i, out, True, None, None, 0.0, 0, deterministic())
                    grads_ab[2 * i + 1] = out.to(b.dtype) if ret else None
                    if not ret:
                        _notify_grad_ready(ctx.ab_refs[2 * i + 1])
            else:
                dyi = dy[:, br.c0:br.c1]
                g = (dyi @ bf16_view(b, dy.dtype)) * br.scaling      # [T, r]  = d(xa)
                db = (dyi.t() @ xa_list[i]) * br.scaling             # [n, r]
                key = ctx.keys[i]
                xin = native().dropout_fwd(x, br.dropout, key) if key is not None else x   # regenerate drop(x)
                grads_ab[2 * i] = (g.t() @ xin).to(a.dtype)
                grads_ab[2 * i + 1] = db.to(b.dtype)
            g_list.append(g)
        dx = None
        if ctx.needs_input_grad[0]:
            fold = [i for i in range(nb) if ctx.keys[i] is None]
            ext_a = ext_b = None

            def fold_ext():   # no-dropout adapters' dx terms as an extra K-slice of the dX GEMM
                if not fold:
                    return None, None
                ea = _pad_cols(torch.cat([g_list[i].to(dy.dtype) for i in fold], 1))
                eb = torch.cat([bf16_view(ab[2 * i], dy.dtype) for i in fold], 0)            # [R, K]
                return ea, F.pad(eb, (0, 0, 0, ea.shape[1] - eb.shape[0])).t().contiguous()  # [K, Rp]
            wb = ctx.wdq if ctx.wdq is not None else (base if not dense else weight)
            pair_ok = (ctx.pair and all(k is not None for k in ctx.keys) and not deterministic()
                       and ctx.needs_input_grad[5] and ctx.needs_input_grad[7])
            if pair_ok and _DX_C and ctx.masks is not None and not fold and dy.shape[0] >= _MIN_M:
                # the LoRA input-gradient term written once (lora_dx2, from the stored keep bits) and
                # added by the dX GEMM as its C matrix; dA from x in a separate launch — no
                # read-modify-write pass over dx (lora_acc2)
                a0, a1 = bf16_view(ab[0], dy.dtype), bf16_view(ab[2], dy.dtype)
                p0, p1 = branches[0].dropout, branches[1].dropout
                fused_ok = wb.shape[1] % 128 == 0 and all(g.shape[1] % 8 == 0 and g.shape[1] <= 32 for g in g_list)
                if fused_ok and isinstance(wb, torch.Tensor) and _g4w_ok(dy, wb, True):
                    # the masked LoRA input gradient inside the dX GEMM's epilogue (no lora_dx2 matrix)
                    _count("gemm4w")
                    dx = native().gemm4w_loradx(dy, wb, None, 0, g_list, [a0, a1], ctx.masks, [p0, p1])
                elif fused_ok and isinstance(wb, NF4Weight) and _w4_ok(dy, wb, True):
                    codes, sc = wb.g4w_pack()
                    _count("gemm4w-nf4")
                    dx = native().gemm4w_loradx(dy, codes, sc, wb.shape[1], g_list, [a0, a1], ctx.masks, [p0, p1])
                else:
                    c = native().lora_dx2(g_list[0], g_list[1], a0, a1, ctx.masks, p0, p1)
                    dx = _base_gemm_t(dy, wb, None, None, c)
                    del c
                if done_quad is not None:
                    (o0, ret0), (o1, ret1) = done_quad
                else:
                    (o0, ret0), (o1, ret1) = dest(0), dest(2)
                    native().lora_dA_pair(g_list[0], g_list[1], x, o0, o1, ctx.masks, p0, p1)
                ctx.masks = None
                for i, (o, ret) in ((0, (o0, ret0)), (1, (o1, ret1))):
                    if ret:
                        grads_ab[2 * i] = o.to(ab[2 * i].dtype)
                    else:
                        _notify_grad_ready(ctx.ab_refs[2 * i])
                pair_ok = False
                done_dA = True
            else:
                assert done_quad is None, "lora_acc_quad ran but the keep-bit dX path did not"
                ext_a, ext_b = fold_ext()
                dx = _base_gemm_t(dy, wb, ext_a, ext_b)
                done_dA = False
        else:
            pair_ok = done_dA = False
        ctx.wdq = None
        ctx.bts = None
        if done_dA:
            branches_acc = ()
        elif (ctx.pair and dx is not None and all(k is not None for k in ctx.keys) and not deterministic()
                and ctx.needs_input_grad[5] and ctx.needs_input_grad[7]):
            # both adapters' dA and their dx terms in ONE pass over x and dx (lora_acc2)
            (o0, ret0), (o1, ret1) = dest(0), dest(2)
            native().lora_acc2(g_list[0], g_list[1], x, dx, bf16_view(ab[0], dy.dtype), bf16_view(ab[2], dy.dtype),
                               o0, o1, branches[0].dropout, ctx.keys[0], branches[1].dropout, ctx.keys[1], ctx.masks)
            ctx.masks = None
            for i, (o, ret) in ((0, (o0, ret0)), (1, (o1, ret1))):
                if ret:
                    grads_ab[2 * i] = o.to(ab[2 * i].dtype)
                else:
                    _notify_grad_ready(ctx.ab_refs[2 * i])
            branches_acc = ()
        else:
            branches_acc = branches
        for i, br in enumerate(branches_acc):
            key = ctx.keys[i]
            if fast:   # dA += gᵀ·D(x) and (dropout branches) dx += D(g·A), one pass over x / dx
                upd = dx if (dx is not None and key is not None) else None
                if ctx.needs_input_grad[5 + 2 * i] or upd is not None:
                    out, ret = dest(2 * i)
                    native().lora_acc(g_list[i], x, 0, x.shape[1], out, False, upd,
                                      bf16_view(ab[2 * i], dy.dtype) if upd is not None else None,
                                      br.dropout if key is not None else 0.0, key or 0, deterministic())
                    grads_ab[2 * i] = out.to(ab[2 * i].dtype) if (ret and ctx.needs_input_grad[5 + 2 * i]) else None
                    if not ret and ctx.needs_input_grad[5 + 2 * i]:
                        _notify_grad_ready(ctx.ab_refs[2 * i])
            elif dx is not None and key is not None:   # LoRA input grad through the regenerated dropout mask
                native().dropout_bwd_add(dx, g_list[i] @ bf16_view(ab[2 * i], dy.dtype), br.dropout, key)
        dres = dy if ctx.has_residual else None
        dw = None
        if dense and weight is not None and ctx.needs_input_grad[2]:
            dw = (dy.t() @ x).to(weight.dtype)
        dbias = dy.sum(0) if ctx.needs_input_grad[3] else None
        return (dx, dres, dw, dbias, None, *grads_ab)


def _multi_backward(ctx, dy, x, weight, xa_list, base, branches, dense, dest):
    """Backward of 1-4 adapters through the multi-adapter kernels (see ``_multi_ok``): 3 LoRA launches
    (g, dB + dA, and the dX term when it cannot ride in the dX GEMM's prologue)."""
    ab = ctx.ab_refs
    nb = len(branches)
    grads_ab = [None] * (2 * nb)
    masks, ctx.masks = ctx.masks, None
    ps = [br.dropout if k is not None else 0.0 for br, k in zip(branches, ctx.keys)]
    g_list = native().lora_proj_cols(dy, [br.c0 for br in branches], ctx.bts, [br.scaling for br in branches])
    ctx.bts = None
    jobs, fin = [], []
    for i, br in enumerate(branches):
        if ctx.needs_input_grad[5 + 2 * i + 1]:      # dB_i [n_i, r] += dy_iᵀ·xa_i
            o, ret = dest(2 * i + 1)
            jobs.append((xa_list[i], dy, br.c0, br.c1 - br.c0, o, True, -1, 0.0))
            fin.append((2 * i + 1, o, ret))
    for i, br in enumerate(branches):
        if ctx.needs_input_grad[5 + 2 * i]:          # dA_i [r, K] += g_iᵀ·D_i(x)
            o, ret = dest(2 * i)
            jobs.append((g_list[i], x, 0, x.shape[1], o, False, i, ps[i]))
            fin.append((2 * i, o, ret))
    if jobs:
        cols = list(zip(*jobs))
        native().lora_acc_jobs(list(cols[0]), list(cols[1]), list(cols[2]), list(cols[3]), list(cols[4]),
                               list(cols[5]), masks, list(cols[6]), list(cols[7]))
    for idx, o, ret in fin:
        if ret:
            grads_ab[idx] = o.to(ab[idx].dtype)
        else:
            _notify_grad_ready(ab[idx])
    dx = None
    if ctx.needs_input_grad[0]:
        wb = ctx.wdq if ctx.wdq is not None else (base if not dense else weight)
        a_list = [bf16_view(ab[2 * i], dy.dtype) for i in range(nb)]
        if masks is None:    # no dropout: the adapters' g·A as an extra K-slice of the dX GEMM
            ea = _pad_cols(torch.cat([g.to(dy.dtype) for g in g_list], 1))
            eb = torch.cat(a_list, 0)
            dx = _base_gemm_t(dy, wb, ea, F.pad(eb, (0, 0, 0, ea.shape[1] - eb.shape[0])).t().contiguous())
        else:
            fused = nb <= 2 and wb.shape[1] % 128 == 0 and all(g.shape[1] == g_list[0].shape[1] for g in g_list)
            if fused and isinstance(wb, torch.Tensor) and _g4w_ok(dy, wb, True):
                _count("gemm4w")
                dx = native().gemm4w_loradx(dy, wb, None, 0, g_list, a_list, masks, ps)
            elif fused and isinstance(wb, NF4Weight) and _w4_ok(dy, wb, True):
                codes, sc = wb.g4w_pack()
                _count("gemm4w-nf4")
                dx = native().gemm4w_loradx(dy, codes, sc, wb.shape[1], g_list, a_list, masks, ps)
            else:
                c = native().lora_dxc(g_list, a_list, masks, ps)
                dx = _base_gemm_t(dy, wb, None, None, c)
                del c
    ctx.wdq = None
    dres = dy if ctx.has_residual else None
    dw = (dy.t() @ x).to(weight.dtype) if (dense and weight is not None and ctx.needs_input_grad[2]) else None
    dbias = dy.sum(0) if ctx.needs_input_grad[3] else None
    return (dx, dres, dw, dbias, None, *grads_ab)


def _reference(x, base, bias, branches, residual, training):
    w = dequantize_nf4(base, x.dtype) if isinstance(base, NF4Weight) else base
    y = x @ w.to(x.dtype).t()
    if branches:
        extra = torch.zeros_like(y)
        for br in branches:
            xd = F.dropout(x, br.dropout, training=training) if br.dropout > 0 else x
            upd = (xd @ br.a.to(x.dtype).t()) @ br.b.to(x.dtype).t() * br.scaling
            extra = extra.index_add(1, torch.arange(br.c0, br.c1, device=x.device), upd)
        y = y + extra
    if bias is not None:
        y = y + bias
    if residual is not None:
        y = y + residual
    return y


def fused_linear(x: torch.Tensor, base, bias: torch.Tensor | None = None,
                 branches: list[LoraBranch] | tuple = (), residual: torch.Tensor | None = None,
                 training: bool = True) -> torch.Tensor:
    """x [..., K] → [..., N].  See module docstring."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    res2 = residual.reshape(-1, residual.shape[-1]) if residual is not None else None
    if use_native(x2) and x2.dtype == torch.bfloat16:
        weight = None if isinstance(base, NF4Weight) else base
        ab = []
        for br in branches:
            ab += [br.a, br.b]
        y = _FusedLinearFn.apply(x2.contiguous(), None if res2 is None else res2.contiguous(),
                                 weight, bias, (base, tuple(branches), training), *ab)
    else:
        _count("library")
        y = _reference(x2, base, bias, branches, res2, training)
    return y.view(*shape[:-1], y.shape[-1])
