"""Activation checkpointing that replays the same LoRA dropout masks, NF4-aware, with a selective policy
(the reference's ``gradient_checkpointing_enable(gradient_checkpointing_kwargs=...)``,
``Fine-Tuning/qwen3-8b-qlora-dist.py:162-163``), and the host-side dropout key stream the fused LoRA kernels
draw their masks from (``next_dropout_key`` / ``seed_dropout``).  On the HIP path the ``use_reentrant=False`` form
is a lean frame (``_Frame``) with torch's early stop (``tail_skippable``); ops ask ``saves_discarded`` to skip
tensors they would only compute to save in a first forward whose saves are dropped.
"""
from __future__ import annotations

import os

import torch

from .gemm import _IN_CKPT

_KEY = [0x5DEECE66D << 20]

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
        return ckpt.checkpoint(run, *args, use_reentrant=True, preserve_rng_state=_torch_rng_used(args))
    if _torch_rng_used(args):
        # off the HIP path (CPU / LIPA_REFERENCE=1) an op of the layer draws from torch's RNG (F.dropout): torch's
        # implementation, with its RNG snapshot around the recompute
        return ckpt.checkpoint(run, *args, use_reentrant=False)
    return _nonreentrant(run, args)


class _Frame:
    """One checkpointed call in the non-reentrant form (``use_reentrant=False`` semantics, as
    ``torch.utils.checkpoint`` implements them): the forward runs with autograd on, but every tensor an op saves
    for backward is replaced by its index (``pack``); the first ``unpack`` in backward re-runs the layer with the
    same inputs under hooks that collect the saved tensors in the same order, and each unpack hands one over
    (and drops it: a second backward through a retained graph recomputes again).  Gradients flow through the
    ORIGINAL graph — inputs that do not require grad, ``torch.autograd.grad`` and partial backwards work as with
    torch's form.  Like torch's form (early stop, on by default) the recompute does not produce what no saved tensor
    depends on: an op whose output only later ops consume asks :func:`tail_skippable` and, when the first forward
    packed nothing after it, skips that output in the recompute (the decoder layer's down projection — its
    output is the layer output, which the recompute discards).  What is left out is the generality this stack does
    not use (nested checkpoints, pytree inputs, torch-RNG replay — the HIP path's dropout comes from the key
    stream ``checkpoint`` restores) and with it most of the per-layer host time of the reference-faithful step
    (profiles/r6/)."""
    __slots__ = ("run", "args", "count", "saved", "rec", "tails", "tail", "skip")

    def __init__(self, run, args):
        self.run, self.args, self.count, self.saved = run, args, 0, None
        self.rec, self.tails, self.tail, self.skip = None, 0, None, False

    def pack(self, t):
        i = self.count
        self.count += 1
        return i

    def unpack(self, i):
        if self.saved is None or self.saved[i] is None:
            self._recompute()
        t = self.saved[i]
        self.saved[i] = None
        return t

    def _recompute(self):
        rec: list = []
        args = tuple(a.detach().requires_grad_(a.requires_grad) if isinstance(a, torch.Tensor) else a
                     for a in self.args)
        prev = _FRAME[0]
        self.rec, self.tails, _FRAME[0] = rec, 0, self
        try:
            with torch.enable_grad(), torch.autograd.graph.saved_tensors_hooks(_Frame._keep(rec), _Frame._give(rec)):
                self.run(*args)
        finally:
            self.rec, _FRAME[0] = None, prev
        if len(rec) != self.count:
            raise RuntimeError(f"checkpoint recompute saved {len(rec)} tensors, the forward {self.count}: the layer "
                               "took a different code path in the recompute")
        self.saved = rec

    @staticmethod
    def _keep(rec):
        def pack(t):
            rec.append(t)
            return None
        return pack

    @staticmethod
    def _give(rec):
        def unpack(_):   # (the recomputed graph is never backpropagated)
            raise RuntimeError("checkpoint: the recomputed graph is not differentiable")
        return unpack


# the _Frame whose first forward or recompute is running (non-reentrant HIP path), else None
_FRAME: list = [None]


def tail_skippable(n_saves: int) -> bool:
    """Asked by an op right before it computes an output that only LATER ops consume, with the number of tensors
    the op itself saves for backward.  In a checkpointed first forward it records its position (pack count and
    call ordinal) and returns False; in the recompute it returns True for the call at that position when the
    first forward packed nothing after this op's own saves — then no saved tensor depends on the output and the
    op may leave it uncomputed (torch's non-reentrant checkpoint stops its recompute at the last saved tensor)."""
    f = _FRAME[0]
    if f is None:
        return False
    f.tails += 1
    if f.rec is None:                                   # the first forward
        f.tail = (f.tails, f.count, n_saves)
        return False
    return f.skip and f.tail[0] == f.tails and f.tail[1] == len(f.rec)


def saves_discarded() -> bool:
    """True inside the first forward of a lean non-reentrant checkpoint: every tensor saved for backward is dropped
    (the recompute produces it again), so an op may skip materialising a tensor it computes ONLY to save it — it
    must still save a placeholder in its place, so the pack count matches the recompute's."""
    f = _FRAME[0]
    return f is not None and f.rec is None and not _sac_recording()


def _nonreentrant(run, args):
    frame = _Frame(run, args)
    prev = _FRAME[0]
    _FRAME[0] = frame
    try:
        with torch.autograd.graph.saved_tensors_hooks(frame.pack, frame.unpack):
            out = run(*args)
    finally:
        _FRAME[0] = prev
    t = frame.tail
    frame.skip = t is not None and t[0] == frame.tails and t[1] + t[2] == frame.count
    return out


def _torch_rng_used(args) -> bool:
    """Whether a checkpointed layer on these inputs draws from torch's RNG: only off the HIP path (CPU tensors or
    LIPA_REFERENCE=1, where LoRA / attention dropout are torch ops)."""
    from ._native import force_reference
    x = next((a for a in args if isinstance(a, torch.Tensor)), None)
    return x is None or not x.is_cuda or force_reference()



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
