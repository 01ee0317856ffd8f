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
                  ``paged_adamw_8bit`` state format]; "paged" (unified-memory spill) is not
                  needed with 288 GB HBM, so states stay resident on the device.
On CPU both fall back to a reference implementation (used by tests / minigpt).
"""
from __future__ import annotations

import math

import torch

from ..ops import reference as ref
from ..ops._native import native, use_native


class FlatParams:
    """Flatten parameters into one fp32 master buffer + one fp32 grad buffer."""

    def __init__(self, params: list[torch.nn.Parameter], align: int = 64):
        self.params = [p for p in params if p.requires_grad]
        assert self.params, "no trainable parameters"
        dev = self.params[0].device
        self.offsets = []
        n = 0
        for p in self.params:
            self.offsets.append(n)
            n += (p.numel() + align - 1) // align * align
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
        # pointer compare only: slicing a view of the flat buffer per parameter cost ~3 us each
        # (0.2-0.4 ms of host time per step with 144 LoRA tensors, visible as GPU idle)
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
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm: float = 0.0):
        params = list(params)
        if params and isinstance(params[0], dict):   # param groups: single group supported
            group = params[0]
            params = list(group["params"])
            lr = group.get("lr", lr)
            weight_decay = group.get("weight_decay", weight_decay)
        self.flat = FlatParams(params)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        dev = self.flat.data.device
        self.norm_out = torch.zeros(3, dtype=torch.float32, device=dev)   # [norm, clip coef, sumsq]
        self.skip_flag = None                                             # fp16 overflow flag (device)
        self.param_groups = [{"params": self.flat.params, "lr": lr, "weight_decay": weight_decay}]

    # torch.optim-like surface ----------------------------------------------------
    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @property
    def grad_buffer(self) -> torch.Tensor:
        return self.flat.grad

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 norm of the flat grads + clip coefficient, on the device."""
        self.max_grad_norm = max_norm
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
        self.flat.sync_grads()
        self.step_count += 1
        b1, b2 = self.betas
        g = self.flat.grad
        clip = self.norm_out if self.max_grad_norm > 0 else None
        if use_native(g):
            native().adamw(self.flat.data, g, self.exp_avg, self.exp_avg_sq, self._sync_low(), self._lr(), b1, b2,
                           self.eps, self.weight_decay, self.step_count, clip, self.skip_flag)
        else:
            if self.skip_flag is not None and self.skip_flag.item() != 0:
                return
            gg = g * (self.norm_out[1] if clip is not None else 1.0)
            ref.adamw_step(self.flat.data, gg, self.exp_avg, self.exp_avg_sq, self.step_count, self._lr(), b1, b2,
                           self.eps, self.weight_decay)
            if self.flat.mixed:
                self.flat.low.copy_(self.flat.data)


class AdamW8bit(_FlatOptimizer):
    """Blockwise (256) 8-bit AdamW — ``optim="paged_adamw_8bit"`` / ``"adamw_8bit"``."""

    BLOCK = 256

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=0.0):
        super().__init__(params, lr, betas, eps, weight_decay, max_grad_norm)
        from ..quant.nf4 import create_dynamic_map
        dev = self.flat.data.device
        n = self.flat.numel
        nb = (n + self.BLOCK - 1) // self.BLOCK
        self.code_s = create_dynamic_map(True).to(dev)
        self.code_u = create_dynamic_map(False).to(dev)
        z_s = int(torch.argmin(self.code_s.abs()))
        z_u = int(torch.argmin(self.code_u.abs()))
        self.qm = torch.full((n,), z_s, dtype=torch.uint8, device=dev)
        self.qv = torch.full((n,), z_u, dtype=torch.uint8, device=dev)
        self.am = torch.zeros(nb, dtype=torch.float32, device=dev)
        self.av = torch.zeros(nb, dtype=torch.float32, device=dev)

    def _state(self):
        return {"qm": self.qm, "qv": self.qv, "am": self.am, "av": self.av, "flat_data": self.flat.data}

    @torch.no_grad()
    def step(self, closure=None):
        self.flat.sync_grads()
        self.step_count += 1
        b1, b2 = self.betas
        g = self.flat.grad
        clip = self.norm_out if self.max_grad_norm > 0 else None
        if use_native(g):
            native().adamw8bit(self.flat.data, g, self.qm, self.qv, self.am, self.av, self.code_s, self.code_u,
                               self._sync_low(), self._lr(), b1, b2, self.eps, self.weight_decay, self.step_count,
                               clip, self.skip_flag)
            return
        # reference: dequantise states, fp32 update, requantise blockwise
        n, B = self.flat.numel, self.BLOCK
        pad = (-n) % B
        blk = lambda t: torch.cat([t, t.new_zeros(pad)]).view(-1, B)  # noqa: E731
        m = (self.code_s[self.qm.long()].view(-1) if not pad else self.code_s[self.qm.long()])
        m = blk(m) * self.am[:, None]
        v = blk(self.code_u[self.qv.long()]) * self.av[:, None]
        gg = blk(g * (self.norm_out[1] if clip is not None else 1.0))
        p = blk(self.flat.data)
        p.mul_(1 - self._lr() * self.weight_decay)
        m.mul_(b1).add_(gg, alpha=1 - b1)
        v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
        bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
        p.addcdiv_(m, (v / bc2).sqrt().add_(self.eps), value=-self._lr() / bc1)
        self.flat.data.copy_(p.view(-1)[:n])
        self.am.copy_(m.abs().amax(1))
        self.av.copy_(v.amax(1))
        from ..quant.nf4 import _nearest
        self.qm.copy_(_nearest((m / self.am[:, None].clamp_min(1e-30)).view(-1)[:n], self.code_s))
        self.qv.copy_(_nearest((v / self.av[:, None].clamp_min(1e-30)).view(-1)[:n], self.code_u))
        if self.flat.mixed:
            self.flat.low.copy_(self.flat.data)
        elif self.flat.shadow is not None:
            self.flat.shadow.copy_(self.flat.data)


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
            g["lr"] = lr

    def step(self):
        self.last_step += 1
        self._apply()

    def get_last_lr(self):
        return [self.opt.param_groups[0]["lr"]]

    def state_dict(self):
        return {"last_step": self.last_step}

    def load_state_dict(self, sd):
        self.last_step = sd["last_step"]
        self._apply()
