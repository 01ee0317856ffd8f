"""Fused AdamW optimizers over flat parameter / gradient buffers.

The trainable set is flattened ONCE: every trainable parameter's ``.data`` and ``.grad``
become views into contiguous fp32 buffers.  Consequences (all MI355X-motivated):
  * an optimizer step is 2-3 kernel launches for the whole model (grad-norm, clip coef and
    the update stay on the device — no host sync per step);
  * the flat gradient buffer IS the communication buffer: DDP all-reduces / ZeRO
    reduce-scatters it directly over RCCL without packing;
  * gradient accumulation accumulates in place (autograd adds into existing ``.grad``).

``AdamW``       — torch.optim.AdamW semantics (``optim="adamw_torch"``).
``AdamW8bit``   — blockwise 8-bit states with the dynamic maps [ext: bitsandbytes
                  ``paged_adamw_8bit`` state format].  ``paged="host"`` (or ``LIPA_PAGED_OPTIM=host``)
                  places the states in pinned, device-mapped host memory: the update kernel reads and
                  writes them across the host link and they take no HBM (bitsandbytes pages its states
                  to the host under memory pressure; with 288 GB of HBM the default keeps them resident).
On CPU both fall back to a reference implementation (used by tests / minigpt).
"""
from __future__ import annotations

import math

import torch

from ..ops import reference as ref
from ..ops._native import native, use_native
from ..ops.linear import nf4_cache_advance



class FlatParams:
    """Flatten parameters into one fp32 master buffer + one fp32 grad buffer.

    ``groups`` (optional) partitions ``params`` into optimizer param groups; each group is a
    contiguous segment of the flat buffers starting on a ``seg_align`` boundary, so a per-group
    update is one kernel launch over a slice (the 8-bit optimizer's 256-element state blocks
    never straddle two groups)."""

    def __init__(self, params: list[torch.nn.Parameter], align: int = 64, groups: list[list] | None = None,
                 seg_align: int = 256):
        if groups is None:
            groups = [list(params)]
        groups = [[p for p in g if p.requires_grad] for g in groups]
        self.params = [p for g in groups for p in g]
        assert self.params, "no trainable parameters"
        dev = self.params[0].device
        self.offsets = []
        self.segments = []                       # [start, end) of each group in the flat buffers
        n = 0
        for g in groups:
            s0 = n
            for p in g:
                self.offsets.append(n)
                n += (p.numel() + align - 1) // align * align
            n = (n + seg_align - 1) // seg_align * seg_align
            self.segments.append((s0, n))
        self.numel = n
        self.data = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.low = None                      # bf16/fp16 model copies, when params are low precision
        low_params = [p for p in self.params if p.dtype != torch.float32]
        if low_params:
            self.low = torch.zeros(n, dtype=low_params[0].dtype, device=dev)
        for p, o in zip(self.params, self.offsets):
            k = p.numel()
            self.data[o:o + k].copy_(p.detach().reshape(-1).float())
            if p.dtype == torch.float32:
                p.data = self.data[o:o + k].view_as(p)
            else:
                self.low[o:o + k].copy_(p.detach().reshape(-1))
                p.data = self.low[o:o + k].view_as(p)
            p.grad = self.grad[o:o + k].view_as(p) if p.dtype == torch.float32 else None
            p._lipa_flat_grad = p.dtype == torch.float32   # kernels may accumulate into p.grad in place
        self.mixed = self.low is not None
        self.grad_ptrs = [self.grad[o:o + p.numel()].data_ptr() for p, o in zip(self.params, self.offsets)]
        # bf16 shadows of fp32 params (LoRA adapters): refreshed by the update kernel itself,
        # consumed by the fused GEMMs — no per-forward fp32→bf16 conversion kernels
        self.shadow = None
        if not self.mixed and dev.type == "cuda":
            self.shadow = self.data.to(torch.bfloat16)
            for p, o in zip(self.params, self.offsets):
                p._lipa_shadow = self.shadow[o:o + p.numel()].view_as(p)

    def sync_grads(self):
        """Copy grads that autograd allocated separately (low-precision params) into the flat
        buffer.  fp32 params accumulate straight into their views."""
        # pointer compare only: slicing a view of the flat buffer per parameter cost ~3 us each (an fp32
        # param's grad is separate only after something set it to None, e.g. zero_grad(set_to_none=True))
        for p, o, ptr in zip(self.params, self.offsets, self.grad_ptrs):
            g = p.grad
            if g is None or g.data_ptr() == ptr:
                continue
            self.grad[o:o + p.numel()].add_(g.reshape(-1).float())
            p.grad = None

    def zero_grad(self):
        self.grad.zero_()
        for p in self.params:
            if p.dtype != torch.float32:
                p.grad = None


class _FlatOptimizer:
    """Base of the fused flat-buffer optimizers.  ``params`` is an iterable of parameters or of
    torch-style param-group dicts (``{"params": [...], "lr": ..., "weight_decay": ...}``, e.g. the
    decay / no-decay split of ``temp/ddp_gpt_wikitext2.py:337-344``); every group keeps its own lr
    and weight decay and is updated as one contiguous segment of the flat buffers."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm: float = 0.0):
        params = list(params)
        if params and isinstance(params[0], dict):
            groups = [dict(g) for g in params]
        else:
            groups = [{"params": params}]
        for g in groups:
            g["params"] = [p for p in g["params"] if p.requires_grad]
            g.setdefault("lr", lr)
            g.setdefault("weight_decay", weight_decay)
            g.setdefault("initial_lr", g["lr"])
        groups = [g for g in groups if g["params"]]
        self.flat = FlatParams([p for g in groups for p in g["params"]], groups=[g["params"] for g in groups])
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        dev = self.flat.data.device
        self.norm_out = torch.zeros(3, dtype=torch.float32, device=dev)   # [norm, clip coef, sumsq]
        self.skip_flag = None                                             # fp16 overflow flag (device)
        self.param_groups = groups

    def _segments(self):
        """(start, end, lr, weight_decay) per param group."""
        for (s0, s1), g in zip(self.flat.segments, self.param_groups):
            yield s0, s1, float(g["lr"]), float(g["weight_decay"])

    # torch.optim-like surface ----------------------------------------------------
    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()
        # a clip_grad_norm_ that no step() followed (a logged-only norm, a skipped step) must not let the next
        # step() skip its own sync_grads / NF4-cache release
        self._prepared = False

    @property
    def grad_buffer(self) -> torch.Tensor:
        return self.flat.grad

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 norm of the flat grads + clip coefficient, on the device.  The host-side step preparation
        (separately allocated grads folded into the flat buffer — which the norm must include — and the NF4
        expansion cache released) runs here, before the norm launches, so step() is one launch per group
        right behind them."""
        self.max_grad_norm = max_norm
        nf4_cache_advance()
        self.flat.sync_grads()
        self._prepared = True    # step() right behind: no second pass over the parameters
        g = self.flat.grad
        if use_native(g):
            native().grad_norm(g, float(max_norm), self.norm_out, False)
        else:
            n = g.norm()
            self.norm_out[0] = n
            self.norm_out[1] = min(1.0, max_norm / (n.item() + 1e-6)) if max_norm > 0 else 1.0
        return self.norm_out[0]

    def state_dict(self) -> dict:
        return {"step": self.step_count, "lr": self.lr, "state": {k: v for k, v in self._state().items()}}

    def load_state_dict(self, sd: dict):
        self.step_count = sd["step"]
        self.lr = sd.get("lr", self.lr)
        st = self._state()
        for k, v in sd["state"].items():
            st[k].copy_(v)
        if self.flat.mixed:
            self.flat.low.copy_(self.flat.data)
        elif self.flat.shadow is not None:
            self.flat.shadow.copy_(self.flat.data)

    def _lr(self):
        return self.param_groups[0]["lr"]

    def _sync_low(self):
        return self.flat.low if self.flat.mixed else self.flat.shadow


class AdamW(_FlatOptimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, max_grad_norm=0.0):
        super().__init__(params, lr, betas, eps, weight_decay, max_grad_norm)
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)

    def _state(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "flat_data": self.flat.data}

    @torch.no_grad()
    def step(self, closure=None):
        if not getattr(self, "_prepared", False):   # (clip_grad_norm_ already did it)
            nf4_cache_advance()
            self.flat.sync_grads()
        self._prepared = False
        self.step_count += 1
        b1, b2 = self.betas
        g = self.flat.grad
        clip = self.norm_out if self.max_grad_norm > 0 else None
        low = self._sync_low()
        if use_native(g):
            for s0, s1, lr, wd in self._segments():
                native().adamw(self.flat.data[s0:s1], g[s0:s1], self.exp_avg[s0:s1], self.exp_avg_sq[s0:s1],
                               None if low is None else low[s0:s1], lr, b1, b2, self.eps, wd, self.step_count,
                               clip, self.skip_flag)
        else:
            if self.skip_flag is not None and self.skip_flag.item() != 0:
                return
            gg = g * (self.norm_out[1] if clip is not None else 1.0)
            for s0, s1, lr, wd in self._segments():
                ref.adamw_step(self.flat.data[s0:s1], gg[s0:s1], self.exp_avg[s0:s1], self.exp_avg_sq[s0:s1],
                               self.step_count, lr, b1, b2, self.eps, wd)
            if self.flat.mixed:
                self.flat.low.copy_(self.flat.data)


class AdamW8bit(_FlatOptimizer):
    """Blockwise (256) 8-bit AdamW — ``optim="paged_adamw_8bit"`` / ``"adamw_8bit"``."""

    BLOCK = 256

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=0.0,
                 paged: str | None = None):
        super().__init__(params, lr, betas, eps, weight_decay, max_grad_norm)
        import os

        from ..quant.nf4 import create_dynamic_map
        dev = self.flat.data.device
        n = self.flat.numel
        nb = (n + self.BLOCK - 1) // self.BLOCK
        self.code_s = create_dynamic_map(True).to(dev)
        self.code_u = create_dynamic_map(False).to(dev)
        z_s = int(torch.argmin(self.code_s.abs()))
        z_u = int(torch.argmin(self.code_u.abs()))
        paged = paged if paged is not None else os.environ.get("LIPA_PAGED_OPTIM", "device")
        if paged not in ("device", "host"):
            raise ValueError(f"paged={paged!r}: 'device' (HBM-resident states) or 'host' (pinned host memory)")
        # the states' placement: HBM, or pinned device-mapped host memory (GPU only; CPU tensors are host memory)
        self.paged = paged if use_native(self.flat.data) else "device"

        def state(numel, dtype, fill):
            if self.paged == "host":
                t = native().host_mapped_empty(numel, dtype)
                return t.fill_(fill)
            return torch.full((numel,), fill, dtype=dtype, device=dev)
        self.qm = state(n, torch.uint8, z_s)
        self.qv = state(n, torch.uint8, z_u)
        self.am = state(nb, torch.float32, 0.0)
        self.av = state(nb, torch.float32, 0.0)

    def _state(self):
        return {"qm": self.qm, "qv": self.qv, "am": self.am, "av": self.av, "flat_data": self.flat.data}

    @torch.no_grad()
    def step(self, closure=None):
        if not getattr(self, "_prepared", False):   # (clip_grad_norm_ already did it)
            nf4_cache_advance()
            self.flat.sync_grads()
        self._prepared = False
        self.step_count += 1
        b1, b2 = self.betas
        g = self.flat.grad
        clip = self.norm_out if self.max_grad_norm > 0 else None
        if use_native(g):
            low = self._sync_low()
            B = self.BLOCK
            for s0, s1, lr, wd in self._segments():
                native().adamw8bit(self.flat.data[s0:s1], g[s0:s1], self.qm[s0:s1], self.qv[s0:s1],
                                   self.am[s0 // B:(s1 + B - 1) // B], self.av[s0 // B:(s1 + B - 1) // B],
                                   self.code_s, self.code_u, None if low is None else low[s0:s1], lr, b1, b2,
                                   self.eps, wd, self.step_count, clip, self.skip_flag)
            return
        # reference: dequantise states, fp32 update, requantise blockwise
        B = self.BLOCK
        lr_e = torch.empty((self.flat.numel + B - 1) // B, 1, dtype=torch.float32, device=g.device)
        wd_e = torch.empty_like(lr_e)
        for s0, s1, lr, wd in self._segments():       # per-block lr / wd of its group
            lr_e[s0 // B:(s1 + B - 1) // B] = lr
            wd_e[s0 // B:(s1 + B - 1) // B] = wd
        adamw8bit_reference(self.flat.data, g * (self.norm_out[1] if clip is not None else 1.0), self.qm, self.qv,
                            self.am, self.av, self.code_s, self.code_u, self.step_count, lr_e, b1, b2, self.eps, wd_e)
        if self.flat.mixed:
            self.flat.low.copy_(self.flat.data)
        elif self.flat.shadow is not None:
            self.flat.shadow.copy_(self.flat.data)


def adamw8bit_reference(p, g, qm, qv, am, av, code_s, code_u, step, lr, b1, b2, eps, wd, block: int = 256):
    """Blockwise 8-bit AdamW step in plain torch (the CPU twin of ``adamw8bit_k``): dequantise the
    signed first / unsigned second moment with their per-block absmax, fp32 update, requantise to
    the nearest dynamic-map code.  ``lr`` / ``wd``: floats or per-block [nb, 1] tensors; ``g`` is
    already clip-scaled.  Updates p, qm, qv, am, av in place."""
    from ..quant.nf4 import _nearest
    n, B = p.numel(), block
    pad = (-n) % B
    blk = lambda t: torch.cat([t, t.new_zeros(pad)]).view(-1, B) if pad else t.view(-1, B)  # noqa: E731
    m = blk(code_s[qm.long()]) * am[:, None]
    v = blk(code_u[qv.long()]) * av[:, None]
    gg = blk(g.float())
    pp = blk(p.float())
    pp.mul_(1 - lr * wd)
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    if isinstance(lr, torch.Tensor):
        pp.add_(m / (v / bc2).sqrt().add_(eps) * (-lr / bc1))
    else:
        pp.add_(m / (v / bc2).sqrt().add_(eps), alpha=-lr / bc1)
    p.copy_(pp.view(-1)[:n])
    am.copy_(m.abs().amax(1))
    av.copy_(v.amax(1))
    qm.copy_(_nearest((m / am[:, None].clamp_min(1e-30)).view(-1)[:n], code_s))
    qv.copy_(_nearest((v / av[:, None].clamp_min(1e-30)).view(-1)[:n], code_u))


def is_8bit(name: str) -> bool:
    """HF ``optim`` names served by the blockwise 8-bit AdamW."""
    return name.lower() in ("paged_adamw_8bit", "adamw_8bit", "adamw_bnb_8bit")


NO_DECAY_DEFAULT = ("bias", "LayerNorm.weight", "norm.weight", "ln_", "ln1", "ln2", "ln_f")


def decay_param_groups(model: torch.nn.Module, weight_decay: float, no_decay=NO_DECAY_DEFAULT) -> list[dict]:
    """The decay / no-decay split of ``temp/ddp_gpt_wikitext2.py:337-344``: parameters whose name
    contains one of ``no_decay`` (biases, LayerNorm weights) get ``weight_decay=0``.  Also puts
    every 1-D parameter (norm scales of our own modules) in the no-decay group."""
    dec, nod = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (nod if (p.ndim < 2 or any(k in n for k in no_decay)) else dec).append(p)
    return [g for g in ({"params": dec, "weight_decay": weight_decay}, {"params": nod, "weight_decay": 0.0})
            if g["params"]]


def build_optimizer(name: str, params, lr: float, weight_decay: float = 0.0, betas=(0.9, 0.999), eps=1e-8,
                    max_grad_norm: float = 1.0):
    """HF ``TrainingArguments.optim`` names → our fused optimizers."""
    name = name.lower()
    if name in ("adamw_torch", "adamw", "adamw_torch_fused", "adamw_hf"):
        return AdamW(params, lr, betas, eps, weight_decay, max_grad_norm)
    if name in ("paged_adamw_8bit", "adamw_8bit", "adamw_bnb_8bit", "paged_adamw_32bit"):
        if name == "paged_adamw_32bit":
            return AdamW(params, lr, betas, eps, weight_decay, max_grad_norm)
        return AdamW8bit(params, lr, betas, eps, weight_decay, max_grad_norm)
    raise ValueError(f"unknown optimizer {name}")


# ------------------------------------------------------------------------------ schedules
class LRScheduler:
    """HF-style schedulers driving ``optimizer.param_groups[0]['lr']``."""

    def __init__(self, optimizer, kind: str, base_lr: float, total_steps: int, warmup_steps: int = 0,
                 min_lr: float = 0.0, gamma: float = 0.95, step_size: int = 1):
        self.opt, self.kind, self.base_lr = optimizer, kind, base_lr
        self.total, self.warmup, self.min_lr = max(1, total_steps), warmup_steps, min_lr
        self.gamma, self.step_size = gamma, step_size
        self.last_step = 0
        self._apply()

    def lr_at(self, s: int) -> float:
        if self.kind == "warmup_lr":            # DeepSpeed WarmupLR (log warmup, then constant)
            if s < self.warmup:
                return self.min_lr + (self.base_lr - self.min_lr) * math.log(s + 1) / math.log(self.warmup)
            return self.base_lr
        if s < self.warmup:
            return self.base_lr * (s + 1) / max(1, self.warmup) if self.kind != "constant" else self.base_lr
        p = (s - self.warmup) / max(1, self.total - self.warmup)
        if self.kind == "linear":
            return self.base_lr * max(0.0, 1.0 - p)
        if self.kind == "cosine":
            return self.min_lr + (self.base_lr - self.min_lr) * 0.5 * (1 + math.cos(math.pi * min(1.0, p)))
        if self.kind == "step":
            return self.base_lr * self.gamma ** (s // self.step_size)
        return self.base_lr

    def _apply(self):
        lr = self.lr_at(self.last_step)
        for g in self.opt.param_groups:
            # a group with its own lr follows the same schedule shape (torch LambdaLR semantics)
            init = g.get("initial_lr", self.base_lr)
            g["lr"] = lr if init == self.base_lr or self.base_lr == 0 else lr * init / self.base_lr

    def step(self):
        self.last_step += 1
        self._apply()

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]

    def state_dict(self):
        return {"last_step": self.last_step}

    def load_state_dict(self, sd):
        self.last_step = sd["last_step"]
        self._apply()
