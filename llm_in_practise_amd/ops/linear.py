"""Frozen-base linear with LoRA branches over NF4 or bf16 bases (K9): the op every
projection of the stack runs through.

    y[:, c0:c1] (+)= x · deq(W)ᵀ  +  Σ_i s_i · (drop_i(x) · A_iᵀ) · B_iᵀ   (+ residual)

* ``base`` is a bf16 ``[N, K]`` tensor (LoRA / full fine-tune) or an :class:`NF4Weight` (QLoRA).  Projections
  that share an input (q|k|v, gate|up) are row-concatenated into one base and one GEMM; each LoRA branch owns a
  column range ``[c0, c1)``.  The base GEMMs themselves are dispatched by ``ops/gemm.py`` (gemm4w, the NF4
  dequant-GEMM or one expansion per step, decode kernels).
* LoRA kernel forms (csrc/kernels/lora.hip, gemm4w_lora.hip), one per adapter layout:
  - pair — q_proj + v_proj of rank <= 8 (the QLoRA configs): ``lora_proj2`` (both s·D(x)·Aᵀ in one pass over x,
    keep bits stored), backward ``lora_proj_pair`` + ``lora_acc_quad`` (both dB and dA in one launch);
  - multi — 1-4 adapters of rank 8 / 16 (BASELINE #2: q, k, v, o): ``lora_proj_m``, ``lora_proj_cols``,
    ``lora_acc_jobs``;
  - per-branch — any other rank <= 16 / 128-aligned shape: ``lora_proj`` / ``lora_acc`` per adapter;
  - general — anything else (rank > 16, odd widths, > 4 adapters): torch matmuls as an extra K-slice of the base
    GEMM.
  At training sizes the adapters' B term rides inside the forward GEMM as extra MFMA K-steps (``gemm4w_lora``)
  and the masked input-gradient term inside the dX GEMM's prologue (``gemm4w_loradx``); at decode / small M the
  B term is added into the adapters' column blocks (``lora_apply``).

Reference parity: PEFT ``LoraConfig(r, lora_alpha, lora_dropout, target_modules)``
(``Fine-Tuning/qwen3-8b-qlora.py:107-114``), scaling = alpha / r.
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn.functional as F

from ..quant.nf4 import NF4Weight, dequantize_nf4
from ._native import env_flag, fn_apply, native, use_native
from .checkpoint import _KEY, _sac_recording, checkpoint, next_dropout_key, sac_put, sac_take, seed_dropout  # noqa: F401
from .gemm import (GEMM_STATS, _MIN_M, _base_gemm, _base_gemm_t, _count, _g4w_ok, _nf4_expand,  # noqa: F401
                   _nf4_w4, _w4_ok, head_logits, nf4_cache_advance)

EXT_ALIGN = 32   # the general form's K-slice: MFMA K-steps of 32


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
    return env_flag("LIPA_DETERMINISTIC") or torch.are_deterministic_algorithms_enabled()


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
    """Shapes the fused LoRA branch kernels (csrc/kernels/lora.hip) take: up to 4 adapters of rank <= 16 on
    128-aligned column ranges of a 128-aligned input (else the general torch form)."""
    K = x.shape[1]
    return (K % 128 == 0 and len(branches) <= 4
            and all(br.a.shape[0] <= 16 and (br.c1 - br.c0) % 128 == 0 for br in branches))


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
        # the fused kernels: the adapters' B term inside gemm4w (epi) or added by lora_apply into ONLY their
        # column blocks of the base GEMM's output; the general form below serves the odd-shaped rest
        apply = fast
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
                # training with dropout on both: keep the masks' bits (2 bits / element of x) for the backward (lora_acc_quad, gemm4w_loradx)
                masks = (torch.empty(2, x.shape[0], x.shape[1] // 8, dtype=torch.uint8, device=x.device)
                         if need_xa and all(k is not None for k in keys) else None)
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
            # the general form: each adapter's s·D(x)·Aᵀ by torch, all of them one extra K-slice of the base GEMM
            N = base.shape[0]
            rtot = sum(br.a.shape[0] for br in branches)
            rp = (rtot + EXT_ALIGN - 1) // EXT_ALIGN * EXT_ALIGN
            layout = tuple((br.c0, br.c1, br.a.shape[0]) for br in branches)
            ext_b = (_zero_buffer(f"lora_b{layout}", N, rp, x) if not torch.cuda.is_current_stream_capturing()
                     else x.new_zeros(N, rp))
            cols, r0 = [], 0
            for br, a, b in zip(branches, ab[0::2], ab[1::2]):
                r = a.shape[0]
                p = br.dropout if training else 0.0
                key = next_dropout_key() if p > 0 else None
                xd = native().dropout_fwd(x, p, key) if key is not None else x
                xa = xd @ bf16_view(a, x.dtype).t()                # [T, r]
                cols.append(xa * br.scaling)
                ext_b[br.c0:br.c1, r0:r0 + r] = bf16_view(b, x.dtype)
                xa_list.append(xa)
                keys.append(key)
                r0 += r
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
                  and all(bt.shape[1] % 512 == 0 for bt in ctx.bts))
        if pair_g:
            g_list = list(native().lora_proj_pair(dy, branches[0].c0, ctx.bts[0], branches[0].scaling,
                                                  branches[1].c0, ctx.bts[1], branches[1].scaling))
            xs = xa_list
            if (ctx.needs_input_grad[6] and ctx.needs_input_grad[8] and not deterministic() and xs[0] is not None
                    and xs[1] is not None and xs[0].stride(0) == xs[1].stride(0) and xs[0].shape[1] <= 8
                    and all((br.c1 - br.c0) % 128 == 0 for br in branches)):
                (o0, ret0), (o1, ret1) = dest(1), dest(3)
                # with the dropout pair's dA due too (the keep-bit path below), both dB and both dA in ONE launch
                quad = (ctx.pair and all(k is not None for k in ctx.keys) and ctx.masks is not None
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
            if pair_ok and ctx.masks is not None and not fold and dy.shape[0] >= _MIN_M:
                # the masked LoRA input-gradient term from the stored keep bits, inside the dX GEMM (or, for shapes
                # gemm4w_loradx does not take, written once by lora_dx2 and added as the GEMM's C matrix); dA by
                # lora_acc_quad above or one lora_dA_pair launch — no read-modify-write pass over dx
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
                done_dA = True
            else:
                assert done_quad is None, "lora_acc_quad ran but the keep-bit dX path did not"
                ext_a, ext_b = fold_ext()
                dx = _base_gemm_t(dy, wb, ext_a, ext_b)
                done_dA = False
        else:
            done_dA = False
        ctx.wdq = None
        ctx.bts = None
        ctx.masks = None
        # dA (and, for dropout adapters outside the fused dX paths, their input-gradient term) per adapter
        branches_acc = () if done_dA else branches
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
        y = fn_apply(_FusedLinearFn, x2.contiguous(), None if res2 is None else res2.contiguous(),
                                 weight, bias, (base, tuple(branches), training), *ab)
    else:
        _count("library")
        y = _reference(x2, base, bias, branches, res2, training)
    return y.view(*shape[:-1], y.shape[-1])
