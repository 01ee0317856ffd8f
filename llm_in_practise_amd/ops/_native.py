"""Loader for the in-tree native extensions.

* ``llm_in_practise_amd._C``   — HIP/CDNA4 kernels for gfx950 (``csrc/kernels/*.hip``),
  built by ``python setup.py build_ext --inplace`` (or ``__graft_entry__.build()``).
* ``llm_in_practise_amd._cpu`` — host C++ runtime pieces (CPU AdamW for ZeRO-Offload,
  the token data loader) built with g++.

Dispatch rule used by every op: a CUDA(HIP) tensor runs the native kernel and the op
raises if ``_C`` is missing — there is no silent eager fallback on a GPU box.  CPU tensors
run ``ops/reference.py``.  ``LIPA_REFERENCE=1`` explicitly forces the reference path on
the GPU (used only to produce A/B baselines).
"""
from __future__ import annotations

import importlib
import os

import torch

_C = None
_CPU = None
_ERR: Exception | None = None


class NativeMissing(RuntimeError):
    pass


def native():
    """Return the HIP extension module, raising loudly if it is not built."""
    global _C, _ERR
    if _C is None:
        try:
            _C = importlib.import_module("llm_in_practise_amd._C")
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
            raise NativeMissing(
                "HIP extension llm_in_practise_amd._C is not built (or failed to load: "
                f"{e}). Run `python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).") from e
    return _C


def has_native() -> bool:
    try:
        native()
        return True
    except NativeMissing:
        return False


# Per-op environment switches are read on every call (tests and smoke() flip them at run time), but through
# os.environ's encoded mapping: os.environ.get() encodes the key each time (~1.5 us, ~1k calls per step)
def env_flag(name: str) -> bool:
    """``os.environ.get(name) == "1"`` at a fraction of its cost (CPython's os.environ keeps the encoded
    environment in ``_data``; any other mapping takes the plain path)."""
    data = getattr(os.environ, "_data", None)
    if data is not None:
        return data.get(name.encode()) == b"1"
    return os.environ.get(name) == "1"


def force_reference() -> bool:
    return env_flag("LIPA_REFERENCE")


_Function = torch.autograd.Function
_functorch_active = torch._C._are_functorch_transforms_active


def fn_apply(fn, *args):
    """``fn.apply(*args)`` for the ops' autograd Functions without torch's Python prologue: ``Function.apply``
    binds default arguments when ``setup_context`` is overridden (none of these Functions does) and passes every
    argument through functorch's dead-wrapper unwrap — 5-8 us per call at 10-25 arguments, ~500 calls in a
    reference-faithful step.  Under functorch transforms (vmap / grad) the full path runs."""
    if _functorch_active():
        return fn.apply(*args)
    return super(_Function, fn).apply(*args)


def use_native(*tensors: torch.Tensor | None) -> bool:
    """True when the op must run on the HIP kernels."""
    for t in tensors:
        if t is not None and isinstance(t, torch.Tensor):
            if t.is_cuda and not force_reference():
                native()  # raise if missing
                return True
            return False
    return False


def cpu_native():
    """Host C++ extension (CPU Adam, loaders).  Built in-tree on first use if missing."""
    global _CPU
    if _CPU is None:
        try:
            _CPU = importlib.import_module("llm_in_practise_amd._cpu")
        except ImportError:
            from ..csrc.build import build_cpu_extension
            _CPU = build_cpu_extension()
    return _CPU
