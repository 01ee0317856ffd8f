"""ZeRO-1/2/3 (+ CPU offload) engine with DeepSpeed-config semantics.

One process per GPU; collectives are ``torch.distributed`` (``"nccl"`` = RCCL over xGMI on
MI355X, ``gloo`` on CPU):

* stage 0: gradients all-reduced (DDP-equivalent); replicated optimizer.
* stage 1: gradients all-reduced; optimizer state + fp32 master partitioned — each rank updates
  its contiguous 1/W shard of the flat parameter buffer, then ``all_gather_into_tensor``.
* stage 2: gradients ``reduce_scatter_tensor``-ed straight into the owner's shard (bucketed
  by ``reduce_bucket_size``); grad-norm from shard partial sums + one scalar all-reduce.
* stage 3: parameters partitioned per *unit* (each block of a ModuleList, plus the root).
  ``ds_zero3_config.json`` semantics (``Fine-Tuning/ds_zero3_config.json:13-21``):
    - a unit's full flat weight is all-gathered in its forward pre-hook (or was PREFETCHED: when a
      unit is used, the next units in the recorded execution order are all-gathered
      asynchronously — ``async_op`` RCCL on its own stream — until ``stage3_prefetch_bucket_size``
      parameters are in flight, never exceeding ``stage3_max_live_parameters`` live);
    - after its forward a unit is freed (``resize_(0)``) unless it is persistent
      (``stage3_param_persistence_threshold``) or will be reused by the backward within
      ``stage3_max_reuse_distance`` parameters;
    - a hook on the unit's output gradient re-gathers it for its backward and prefetches the
      units the backward visits next;
    - finished units' gradients are packed rank-major into persistent bucket buffers and
      reduce-scattered asynchronously (``overlap_comm``) in ``reduce_bucket_size`` buckets while
      the backward continues; ``step()`` joins them.
  Frozen NF4 bases stay replicated by default — only trainable parameters and their optimizer
  state are partitioned (QLoRA + ZeRO-3, SURVEY §7.5.3 option 2).  With
  ``zero_optimization.stage3_partition_frozen_quant: true`` (option 1) each unit's quantised bases
  are partitioned too, by whole quant blocks, and all-gathered with its parameters (``_QuantFlat``):
  per-rank base memory 1/W, at one extra byte all-gather of ≈0.53 B/weight per unit use.
* no host synchronisation in ``step()`` (bf16 / fp32): the global-norm clip coefficient stays on
  the device and feeds the fused AdamW kernel.
* checkpoints re-partition on load when the world size changed (per-unit / flat layouts are
  rebuilt from every old rank's shard file).
* ``offload_optimizer: cpu``: fp32 master shard and Adam moments live in (pinned) host memory;
  the update is the native OpenMP/AVX host AdamW (``csrc/cpu/cpu_adam.cpp``); gradients
  stream D2H and the updated compute-dtype shard H2D.
* fp16 ``loss_scale: 0`` → dynamic loss scaling (initial 2^power, window, hysteresis, min);
  bf16 → no scaling.  ``gradient_clipping`` → global-norm clip.

Surface mirrors the DeepSpeed engine the reference drives
(``DeepSpeed-GPTLike-ZeRO-1.py:287-330``): ``engine(x)``, ``engine.backward(loss)``,
``engine.step()`` (steps the optimizer at gradient-accumulation boundaries),
``save_checkpoint(dir, tag)`` / ``load_checkpoint(dir, tag)`` (``<dir>/<tag>/`` with
``mp_rank_00_model_states.pt`` + ``zero_pp_rank_{r}_mp_rank_00_optim_states.pt`` and a
``latest`` file), and :func:`initialize` ≈ ``deepspeed.initialize``.
"""
from __future__ import annotations

import contextlib
import math
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops import reference as ref
from ..ops._native import native, use_native
from ..optim.adamw import LRScheduler
from .dist import COMM, is_dist
from .ds_config import DSConfig, load_ds_config


def _world():
    return dist.get_world_size() if is_dist() else 1


_CHECK = os.environ.get("LIPA_ZERO_CHECK") == "1"     # debug: verify gathered copies / unit grads (host syncs)


def _check(what: str, ok: bool):
    if not ok:
        print(f"[zero-check rank {_rank()}] FAILED: {what}", flush=True)


def _rank():
    return dist.get_rank() if is_dist() else 0


def _pad_to(n, m):
    return (n + m - 1) // m * m


class LossScaler:
    """DeepSpeed-style dynamic fp16 loss scaling (skip / halve with hysteresis / grow per window)."""

    def __init__(self, cfg: DSConfig):
        self.dynamic = cfg.fp16 and cfg.fp16_loss_scale == 0
        self.scale = float(2 ** cfg.fp16_initial_scale_power) if self.dynamic else (cfg.fp16_loss_scale or 1.0)
        self.window, self.hysteresis, self.min_scale = cfg.fp16_loss_scale_window, cfg.fp16_hysteresis, \
            cfg.fp16_min_loss_scale
        self.good_steps, self.cur_hyst = 0, cfg.fp16_hysteresis
        self.enabled = cfg.fp16

    def update(self, overflow: bool):
        if not self.dynamic:
            return
        if overflow:
            self.cur_hyst -= 1
            if self.cur_hyst <= 0:
                self.scale = max(self.min_scale, self.scale / 2)
                self.cur_hyst = self.hysteresis
            self.good_steps = 0
        else:
            self.good_steps += 1
            if self.good_steps % self.window == 0:
                self.scale *= 2
                self.cur_hyst = self.hysteresis


def _in_backward() -> bool:
    """True inside an autograd backward pass (e.g. a reentrant checkpoint's recompute)."""
    try:
        return torch._C._current_graph_task_id() != -1
    except AttributeError:      # pragma: no cover - older torch
        return False


_QALIGN = 512      # bytes: 16 NF4 quant blocks of codes, 512 block scales — shards hold whole blocks


def _frozen_quant_tensors(module: nn.Module, claimed: set) -> tuple[list, list]:
    """(tensors, owners) of the frozen quantised bases under ``module``: every Linear4bit's buffers
    and every fused q|k|v / gate|up NF4 base (models/common.py FusedProjection, whose parts are views
    of it).  ``owners`` are the NF4Weight objects whose derived caches must go when the bytes do."""
    from ..peft.lora import Linear4bit
    from ..quant.nf4 import NF4Weight
    tensors, owners = [], []

    def take(q: NF4Weight):
        owners.append(q)
        for t in q.tensors().values():
            if id(t) not in claimed:
                claimed.add(id(t))
                tensors.append(t)

    for m in module.modules():
        if isinstance(m, Linear4bit) and m.codes.numel():
            take(m.nf4)
        for v in vars(m).values():
            b = getattr(v, "base", None)
            if isinstance(b, NF4Weight) and not isinstance(v, nn.Module):
                take(b)
    return tensors, owners


class _QuantFlat:
    """The frozen quantised bases of one stage-3 unit, partitioned by whole quant blocks (SURVEY.md
    §7.5.3 option 1; ``zero_optimization.stage3_partition_frozen_quant``).

    DeepSpeed stage 3 partitions every module parameter, the frozen 4-bit base included
    (``Fine-Tuning/qwen3-14b-qlora-dist-deepspeed.py:164``, ``Fine-Tuning/ds_zero3_config.json:13-21``).
    Here every storage behind the unit's NF4 tensors (codes, block scales, double-quant scales) is
    laid into ONE uint8 buffer, each segment 512-B aligned, the buffer padded to W × 512 B, and every
    tensor re-pointed (``Tensor.set_``) at its bytes — so the module's buffers, the fused base and the
    parts' views all read the one buffer, and the unit's all-gather / ``resize_(0)`` serves them all.
    Each rank keeps 1/W of the bytes (a whole number of quant blocks); the all-gather is a byte copy,
    so the gathered weight is bit-identical to the unpartitioned one."""

    def __init__(self, tensors, owners, world, rank, device):
        self.tensors, self.owners = tensors, owners
        self.world, self.rank = world, rank
        segs, total = {}, 0
        for t in tensors:
            st = t.untyped_storage()
            k = st.data_ptr()
            if k not in segs:
                segs[k] = (total, st)
                total += _pad_to(max(st.nbytes(), 1), _QALIGN)
        self.npad = _pad_to(max(total, 1), world * _QALIGN)
        self.shard_n = self.npad // world
        full = torch.zeros(self.npad, dtype=torch.uint8, device=device)
        for o, st in segs.values():
            full[o:o + st.nbytes()].copy_(torch.empty(0, dtype=torch.uint8, device=device).set_(st))
        fst = full.untyped_storage()
        with torch.no_grad():
            for t in tensors:
                o = segs[t.untyped_storage().data_ptr()][0]
                t.set_(fst, o // t.element_size() + t.storage_offset(), t.size(), t.stride())
        self.numel = 2 * total          # ≈ quantised weight elements (4-bit codes + their scales)
        self.full = full
        self.shard = full[rank * self.shard_n:(rank + 1) * self.shard_n].clone()

    def drop_caches(self):
        # the g4w-packed copy of the codes goes with them; the decoded fp32 block scales (1/16 of the bf16
        # size) stay cached — rebuilding them at every gather cost more than their bytes (BASELINE #4)
        for q in self.owners:
            q.__dict__.pop("_g4w", None)


def _join(works, kind: str):
    """Join async collectives, timing the wait for the bench's comm record (parallel/dist.py COMM)."""
    ev0 = COMM.events() if torch.cuda.is_available() else None
    t0 = time.perf_counter()
    for w in works:
        w.wait()
    if ev0 is not None:
        COMM.wait_end(kind, ev0)
    elif torch.distributed.get_backend() != "nccl":
        COMM.host_wait(kind, time.perf_counter() - t0)


class _Unit:
    """A stage-3 partition unit: trainable params of one module, flattened and sharded."""

    def __init__(self, name, module, params, world, rank, dtype, device, index=0, block=1):
        self.name, self.module, self.params = name, module, params
        self.index = index
        self.shapes = [p.shape for p in params]
        self.numels = [p.numel() for p in params]
        n = sum(self.numels)
        self.n = n
        self.npad = _pad_to(max(n, 1), world * block)     # block: shards hold whole 8-bit state blocks
        self.shard_n = self.npad // world
        self.world, self.rank = world, rank
        self.dtype, self.device = dtype, device
        full = torch.zeros(self.npad, dtype=dtype, device=device)
        o = 0
        for p, k in zip(params, self.numels):
            full[o:o + k].copy_(p.detach().reshape(-1))
            o += k
        self.shard = full[rank * self.shard_n:(rank + 1) * self.shard_n].clone()
        self.full = full
        self.gathered = True
        self.work = None                  # in-flight async all-gathers (prefetch)
        self.quant: _QuantFlat | None = None
        self._point_params()
        self.grads_ready = 0

    @property
    def size(self) -> int:
        """Elements the unit brings in when gathered (trainable + partitioned frozen quantised)."""
        return self.n + (self.quant.numel if self.quant is not None else 0)

    def _flats(self):
        yield self.full, self.shard
        if self.quant is not None:
            yield self.quant.full, self.quant.shard

    def _point_params(self):
        o = 0
        for p, k, s in zip(self.params, self.numels, self.shapes):
            p.data = self.full[o:o + k].view(s)
            o += k

    @property
    def live(self) -> bool:
        return self.gathered or self.work is not None

    def gather(self, async_op: bool = False) -> bool:
        """All-gather the full weight.  ``async_op``: issue and return (prefetch); a later
        ``gather()`` joins it.  Returns True when a collective was issued."""
        if self.gathered:
            return False
        if self.work is not None:
            if not async_op:
                _join(self.work, "all_gather")
                self.work = None
                self.gathered = True
                self._verify("joined prefetch")
            return False
        works = []
        for full, shard in self._flats():
            full.untyped_storage().resize_(full.numel() * full.element_size())
            if self.world > 1:
                COMM.issue("all_gather", full.numel() * full.element_size())
                w = dist.all_gather_into_tensor(full, shard, async_op=async_op)
                if async_op:
                    works.append(w)
            else:
                full.copy_(shard)
        if works:
            self.work = works
            return True
        self.gathered = True
        self._verify("sync gather")
        return True

    def _verify(self, how: str):
        if not _CHECK:
            return
        for i, (full, shard) in enumerate(self._flats()):
            mine = full.view(self.world, -1)[self.rank]
            _check(f"{self.name} flat {i} ({how}): own slice != shard", bool(torch.equal(mine, shard)))
            if full.is_floating_point():
                _check(f"{self.name} flat {i} ({how}): non-finite", bool(torch.isfinite(full).all()))

    def release(self):
        if self.work is not None:
            _join(self.work, "all_gather")
            self.work = None
            self.gathered = True
        if not self.gathered:
            return
        for full, _ in self._flats():
            full.untyped_storage().resize_(0)
        if self.quant is not None:
            self.quant.drop_caches()
        self.gathered = False


class ZeroEngine:
    def __init__(self, model: nn.Module, config, lr: float | None = None, weight_decay: float | None = None,
                 betas=(0.9, 0.999), eps: float = 1e-8, hidden_size: int | None = None,
                 micro_batch: int | None = None, grad_accum: int | None = None, units: list[nn.Module] | None = None,
                 total_steps: int = 10 ** 9, optim: str | None = None):
        """``optim``: a client optimizer by HF ``TrainingArguments.optim`` name.  ``"paged_adamw_8bit"`` /
        ``"adamw_8bit"`` (``Fine-Tuning/qwen3-14b-qlora-dist-deepspeed.py:151,164``: the client 8-bit
        paged AdamW under ``deepspeed=ds_zero3_config.json``) keeps blockwise-8-bit moments on each
        rank's partition — every shard is a whole number of 256-element state blocks, so the blocks
        (and the update) are the same at any world size; default / ``adamw_torch``: fp32 moments."""
        from ..optim.adamw import is_8bit
        self.world, self.rank = _world(), _rank()
        self.opt8 = bool(optim) and is_8bit(optim)
        self.block = 256 if self.opt8 else 1
        self.optim_name = "paged_adamw_8bit" if self.opt8 else "adamw"
        self.cfg: DSConfig = load_ds_config(config, self.world, micro_batch, grad_accum, hidden_size)
        self.module = model
        self.stage = self.cfg.zero.stage
        opt = (self.cfg.optimizer or {}).get("params", {}) if self.cfg.optimizer else {}
        self.lr = float(opt.get("lr", lr if lr is not None else 1e-3)) if opt.get("lr") != "auto" else float(lr)
        self.wd = float(opt.get("weight_decay", weight_decay if weight_decay is not None else 0.0))
        self.betas = tuple(opt.get("betas", betas))
        self.eps = float(opt.get("eps", eps))
        self.device = next(model.parameters()).device
        self.compute_dtype = torch.bfloat16 if self.cfg.bf16 else torch.float16 if self.cfg.fp16 else None
        if self.compute_dtype is not None:
            for p in model.parameters():
                if p.requires_grad and p.is_floating_point():
                    p.data = p.data.to(self.compute_dtype)
        self.offload = self.cfg.zero.offload_optimizer == "cpu"
        self.scaler = LossScaler(self.cfg)
        self.micro_steps = 0
        self.global_steps = 0
        self.ga = self.cfg.gradient_accumulation_steps
        self.clip = self.cfg.gradient_clipping
        self.last_grad_norm = torch.zeros((), device=self.device)
        self._skipped = 0
        self._sync = True
        params = [p for p in model.parameters() if p.requires_grad]
        # de-duplicate tied params
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        if is_dist():                     # before stage 3 may partition the frozen quantised buffers
            with torch.no_grad():
                for b in model.buffers():
                    dist.broadcast(b, src=0)
        if self.stage == 3:
            self._init_stage3(units)
        else:
            self._init_flat()
        self._init_optimizer_state()
        self.lr_scheduler = self._build_scheduler(total_steps)

    # ------------------------------------------------------------------ layout
    def _init_flat(self):
        W, r = self.world, self.rank
        dtype = self.params[0].dtype
        n = sum(p.numel() for p in self.params)
        self.n = n
        self.npad = _pad_to(n, W * self.block)
        self.shard_n = self.npad // W
        self.flat_model = torch.zeros(self.npad, dtype=dtype, device=self.device)
        self.flat_grad = torch.zeros(self.npad, dtype=torch.float32, device=self.device)
        o = 0
        for p in self.params:
            k = p.numel()
            self.flat_model[o:o + k].copy_(p.detach().reshape(-1))
            p.data = self.flat_model[o:o + k].view_as(p)
            if dtype == torch.float32:
                p.grad = self.flat_grad[o:o + k].view_as(p)
            o += k
        if is_dist():
            dist.broadcast(self.flat_model, src=0)
        if self.stage == 0:               # replicated optimizer (DDP semantics)
            self.shard_n = self.npad
            r = 0
        self.shard_slice = slice(r * self.shard_n, (r + 1) * self.shard_n)
        self.master = self.flat_model[self.shard_slice].float().clone()
        if self.stage == 2:
            self.grad_shard = torch.zeros(self.shard_n, dtype=torch.float32, device=self.device)

    def _init_stage3(self, units):
        W, r = self.world, self.rank
        if units is None:
            units = []
            for m in self.module.modules():
                if isinstance(m, nn.ModuleList):
                    units.extend(list(m))
        unit_of = {}
        for u in units:
            for p in u.parameters():
                if p.requires_grad:
                    unit_of.setdefault(id(p), u)
        groups: dict[int, list] = {}
        order: list = []
        for p in self.params:
            u = unit_of.get(id(p), self.module)
            if id(u) not in groups:
                groups[id(u)] = []
                order.append(u)
            groups[id(u)].append(p)
        if is_dist():
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, src=0)
        self.units = [_Unit(f"u{i}", u, groups[id(u)], W, r, self.params[0].dtype, self.device, index=i,
                            block=self.block) for i, u in enumerate(order)]
        if self.cfg.zero.stage3_partition_frozen_quant and W > 1:   # (world 1: nothing to shard)
            claimed: set = set()
            for u in self.units:
                if u.module is self.module:       # the root unit: its own frozen tensors stay replicated
                    continue
                ts, owners = _frozen_quant_tensors(u.module, claimed)
                if ts:
                    u.quant = _QuantFlat(ts, owners, W, r, self.device)
        self.master = torch.cat([u.shard.float() for u in self.units])
        self.grad_shard = torch.zeros_like(self.master)
        self.unit_offsets, o = [], 0
        for u in self.units:
            self.unit_offsets.append(o)
            o += u.shard_n
        z = self.cfg.zero
        thr = z.stage3_param_persistence_threshold
        self.persistent = {id(u): (u.size < thr or u.module is self.module) for u in self.units}
        self.prefetch_bucket = int(z.stage3_prefetch_bucket_size)
        self.max_live = int(z.stage3_max_live_parameters)
        self.max_reuse = int(z.stage3_max_reuse_distance)
        self.reduce_bucket = max(1, int(z.reduce_bucket_size))
        # ds_config "overlap_comm": True (the reference's ds_zero3_config.json) issues the gradient
        # reduce-scatters asynchronously while the backward continues and prefetches all-gathers ahead of
        # use; False runs every collective synchronously at its point of use (no prefetch, each reduce-scatter
        # joined before the backward goes on) — DeepSpeed's non-overlapped schedule
        self.overlap_comm = bool(z.overlap_comm)
        if not self.overlap_comm:
            self.prefetch_bucket = 0
        self.fwd_order: list[int] = [u.index for u in self.units if u.module is not self.module]
        self._recorded: list[int] = []
        self._recording = True
        self.event_log: list[tuple[str, int]] = []      # ("issue" | "use_fwd" | "use_bwd", unit)
        self.log_events = False
        self._pending_units: list[_Unit] = []
        self._pending_n = 0
        self._bucket = None               # index of the open bucket in _rs_pool
        self._bucket_cap = 0
        self._busy: set[int] = set()      # pool entries whose reduced output is not consumed yet
        self._rs_works: list = []
        self._rs_pool: list = []
        for u in self.units:
            if u.module is not self.module:
                u.module.register_forward_pre_hook(self._pre_fwd(u))
                u.module.register_forward_hook(self._post_fwd(u))
            for p in u.params:
                p.register_post_accumulate_grad_hook(self._grad_hook(u))
        for u in self.units:
            if not self.persistent[id(u)]:
                u.release()

    # ---- stage-3 scheduling -------------------------------------------------------------
    def _log(self, what, u):
        if self.log_events:
            self.event_log.append((what, u.index))

    def _live_params(self) -> int:
        return sum(u.size for u in self.units if u.live)

    def _prefetch(self, seq: list[int], pos: int):
        """Issue async all-gathers for the units after ``pos`` in ``seq`` (prefetch bucket /
        max-live bounded)."""
        if self.prefetch_bucket <= 0:
            return
        budget, live = 0, self._live_params()
        for idx in seq[pos + 1:]:
            u = self.units[idx]
            if budget >= self.prefetch_bucket:
                break
            budget += u.size
            if u.live:
                continue
            if live + u.size > self.max_live:
                break
            if u.gather(async_op=True):
                self._log("issue", u)
            live += u.size

    def _reuse_distance(self, u) -> int:
        """Parameters touched between this unit's forward and its backward (fwd of the later
        units + their bwd)."""
        seq = self.fwd_order
        if u.index not in seq:
            return 1 << 62
        after = seq[seq.index(u.index) + 1:]
        return 2 * sum(self.units[i].size for i in after)

    def _pre_fwd(self, u):
        def hook(mod, args):
            self._log("use_fwd", u)
            u.gather()
            recompute = _in_backward()      # an activation-checkpoint recompute inside the backward
            # the execution order is recorded from the real forward whether or not it builds a graph
            # (reentrant checkpointing runs it under no_grad); a recompute runs the units in reverse
            if self._recording and not recompute and u.index not in self._recorded:
                self._recorded.append(u.index)
            seq = self.fwd_order[::-1] if recompute else self.fwd_order
            if u.index in seq:
                self._prefetch(seq, seq.index(u.index))
        return hook

    def _post_fwd(self, u):
        def hook(mod, args, out):
            if self.persistent[id(u)]:
                return out
            if not torch.is_grad_enabled():
                u.release()
                return out
            t = out[0] if isinstance(out, (tuple, list)) else out
            if isinstance(t, torch.Tensor) and t.requires_grad:
                t.register_hook(self._pre_bwd(u))
            if self._reuse_distance(u) >= self.max_reuse:
                u.release()
            return out
        return hook

    def _pre_bwd(self, u):
        def hook(g):
            self._log("use_bwd", u)
            u.gather()
            seq = self.fwd_order[::-1]
            if u.index in seq:
                self._prefetch(seq, seq.index(u.index))
            return g
        return hook

    def _grad_hook(self, u):
        def hook(p):
            u.grads_ready += 1
            if u.grads_ready == len(u.params):
                u.grads_ready = 0
                self._queue_reduce(u)
        return hook

    def _queue_reduce(self, u):
        """Pack a finished unit's gradients (rank-major) into the open bucket at once — so its
        full weights and grads are freed now — and reduce-scatter the bucket when it is full."""
        W = self.world
        cap = max(1, self.reduce_bucket // max(1, W))
        if self._bucket is not None and self._pending_n + u.shard_n > self._bucket_cap:
            self._flush_reduce()
        if self._bucket is None:
            self._bucket_cap = max(cap, u.shard_n)
            self._bucket = self._rs_buffers(self._bucket_cap)
        bi, _, _ = self._rs_pool[self._bucket]
        view = bi[:W * self._bucket_cap].view(W, self._bucket_cap)
        col = self._pending_n
        flat = torch.zeros(u.npad, dtype=torch.float32, device=self.device)
        o = 0
        for p, k in zip(u.params, u.numels):
            if p.grad is not None:
                flat[o:o + k].copy_(p.grad.reshape(-1))
                p.grad = None
            o += k
        if _CHECK:
            _check(f"{u.name} grads non-finite / huge (max {float(flat.abs().max()):.3g})",
                   bool(torch.isfinite(flat).all()) and float(flat.abs().max()) < 1e3)
        view[:, col:col + u.shard_n].copy_(flat.view(W, u.shard_n))
        self._pending_units.append(u)
        self._pending_n += u.shard_n
        if not self.persistent[id(u)]:
            u.release()
        if self._pending_n >= self._bucket_cap:
            self._flush_reduce()

    def _retire(self, block: bool = False):
        """Fold finished reduce-scatters into the gradient shard and free their buffers
        (``block``: also wait for the oldest one still in flight)."""
        keep = []
        for j, (work, out, units, i) in enumerate(self._rs_works):
            done = work is None or work.is_completed() or (block and j == 0)
            if not done:
                keep.append((work, out, units, i))
                continue
            if work is not None:
                _join([work], "reduce_scatter")
            col = 0
            for u in units:
                o = self.unit_offsets[u.index]
                self.grad_shard[o:o + u.shard_n].add_(out[col:col + u.shard_n], alpha=1.0 / self.world)
                col += u.shard_n
            self._busy.discard(i)
            bi, bo, _ = self._rs_pool[i]
            self._rs_pool[i] = (bi, bo, None)
        self._rs_works = keep

    def _rs_buffers(self, n: int):
        """A persistent (in, out) pair of bucket buffers with room for ``n`` shard elements per
        rank (at most 4 pairs: beyond that the oldest in-flight reduce-scatter is joined)."""
        self._retire()
        while True:
            for i, (bi, bo, work) in enumerate(self._rs_pool):
                if bo.numel() >= n and i not in self._busy:
                    return i
            if len(self._rs_pool) < 4 or not self._rs_works:
                break
            self._retire(block=True)
        free = [i for i in range(len(self._rs_pool)) if i not in self._busy]
        bi = torch.zeros(self.world * n, dtype=torch.float32, device=self.device)
        bo = torch.zeros(n, dtype=torch.float32, device=self.device)
        if free and len(self._rs_pool) >= 4:     # replace a too-small idle pair
            self._rs_pool[free[0]] = (bi, bo, None)
            return free[0]
        self._rs_pool.append((bi, bo, None))
        return len(self._rs_pool) - 1

    def _flush_reduce(self):
        units, n, i = self._pending_units, self._pending_n, self._bucket
        self._pending_units, self._pending_n, self._bucket = [], 0, None
        if not units:
            return
        bi, bo, _ = self._rs_pool[i]
        W, cap = self.world, self._bucket_cap
        src = bi[:W * cap]
        if n < cap:                       # compact the packed columns of a partial bucket
            src = bi[:W * cap].view(W, cap)[:, :n].contiguous().view(-1)
        out = bo[:n]
        work = None
        if W > 1:
            COMM.issue("reduce_scatter", src.numel() * src.element_size())
            work = dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, async_op=self.overlap_comm)
            if not self.overlap_comm:
                work = None          # completed in-line (synchronous schedule); _retire folds it now
        else:
            out.copy_(src[:n])
        self._rs_pool[i] = (bi, bo, work)
        self._busy.add(i)
        self._rs_works.append((work, out, units, i))

    def _join_reduces(self):
        self._flush_reduce()
        while self._rs_works:
            self._retire(block=True)

    # ------------------------------------------------------------------ optimizer state
    def _init_optimizer_state(self):
        dev = torch.device("cpu") if self.offload else self.device
        if self.offload:
            self.master = self.master.cpu().pin_memory() if (self.cfg.zero.pin_memory and torch.cuda.is_available()) \
                else self.master.cpu()
        if self.opt8:      # blockwise 8-bit moments (bitsandbytes dynamic maps) on this rank's partition
            from ..quant.nf4 import create_dynamic_map
            n, nb = self.master.numel(), self.master.numel() // 256
            self.code_s = create_dynamic_map(True).to(dev)
            self.code_u = create_dynamic_map(False).to(dev)
            self.qm = torch.full((n,), int(torch.argmin(self.code_s.abs())), dtype=torch.uint8, device=dev)
            self.qv = torch.full((n,), int(torch.argmin(self.code_u.abs())), dtype=torch.uint8, device=dev)
            self.am = torch.zeros(nb, dtype=torch.float32, device=dev)
            self.av = torch.zeros(nb, dtype=torch.float32, device=dev)
        else:
            self.exp_avg = torch.zeros(self.master.numel(), dtype=torch.float32, device=dev)
            self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.opt_step = 0

    def _build_scheduler(self, total_steps):
        s = self.cfg.scheduler
        if not s:
            return None
        p = s.get("params", {})
        if s.get("type") == "WarmupLR":
            return LRScheduler(self, "warmup_lr", float(p.get("warmup_max_lr", self.lr)), total_steps,
                               int(p.get("warmup_num_steps", 1000)), float(p.get("warmup_min_lr", 0.0)))
        if s.get("type") in ("WarmupDecayLR", "WarmupCosineLR"):
            return LRScheduler(self, "linear" if s["type"] == "WarmupDecayLR" else "cosine",
                               float(p.get("warmup_max_lr", self.lr)), int(p.get("total_num_steps", total_steps)),
                               int(p.get("warmup_num_steps", 0)))
        return None

    @property
    def param_groups(self):
        if not hasattr(self, "_pg"):
            self._pg = [{"lr": self.lr, "weight_decay": self.wd}]
        return self._pg

    # ------------------------------------------------------------------ train-loop surface
    def __call__(self, *a, **kw):
        return self.forward(*a, **kw)

    def forward(self, *a, **kw):
        if self.stage == 3:
            for u in self.units:
                if self.persistent[id(u)]:
                    u.gather()
        return self.module(*a, **kw)

    def train(self, mode=True):
        self.module.train(mode)
        return self

    def eval(self):
        self.module.eval()
        return self

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def is_gradient_accumulation_boundary(self) -> bool:
        return (self.micro_steps + 1) % self.ga == 0

    def backward(self, loss: torch.Tensor):
        scale = self.scaler.scale if self.scaler.enabled else 1.0
        (loss * (scale / self.ga)).backward()
        if self.stage < 3 and self.params[0].dtype != torch.float32:
            o = 0
            for p in self.params:
                k = p.numel()
                if p.grad is not None:
                    self.flat_grad[o:o + k].add_(p.grad.reshape(-1).float())
                    p.grad = None
                o += k

    def step(self):
        boundary = self.is_gradient_accumulation_boundary()
        self.micro_steps += 1
        if not boundary:
            return
        from ..ops.linear import nf4_cache_advance
        nf4_cache_advance()        # the step's NF4 expansions (checkpointed layers) are released
        self._optimizer_step()
        self.global_steps += 1
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()

    def zero_grad(self):
        if self.stage == 3:
            self.grad_shard.zero_()
        else:
            self.flat_grad.zero_()
            if self.stage == 2:
                self.grad_shard.zero_()

    # ------------------------------------------------------------------ the update
    def _reduce_grads(self) -> torch.Tensor:
        """Return this rank's fp32 gradient shard (averaged over ranks)."""
        if self.stage == 3:
            for u in self.units:          # units whose params did not all receive grads
                if u.grads_ready:
                    u.grads_ready = 0
                    self._queue_reduce(u)
            self._join_reduces()
            if _CHECK:
                _check(f"grad shard non-finite / huge (max {float(self.grad_shard.abs().max()):.3g})",
                       bool(torch.isfinite(self.grad_shard).all()) and float(self.grad_shard.abs().max()) < 1e3)
            if self._recording and self._recorded:      # execution order seen by the first step
                self.fwd_order = list(self._recorded)
                self._recording = False
            return self.grad_shard
        if self.stage == 2:
            if self.world > 1:
                dist.reduce_scatter_tensor(self.grad_shard, self.flat_grad, op=dist.ReduceOp.SUM)
                self.grad_shard.div_(self.world)
            else:
                self.grad_shard.copy_(self.flat_grad[self.shard_slice])
            return self.grad_shard
        if self.world > 1:
            dist.all_reduce(self.flat_grad)
            self.flat_grad.div_(self.world)
        return self.flat_grad[self.shard_slice]

    def _global_sumsq(self, g: torch.Tensor) -> torch.Tensor:
        s = g.double().pow(2).sum().float().reshape(1) if g.device.type == "cpu" else g.float().pow(2).sum().reshape(1)
        if self.world > 1 and self.stage > 0:      # stage 0 holds the full replicated gradient
            s = s.to(self.device)
            dist.all_reduce(s)
        return s

    def _optimizer_step(self):
        g = self._reduce_grads()
        inv = 1.0 / self.scaler.scale if self.scaler.enabled else 1.0
        if self.scaler.enabled:           # fp16 dynamic loss scaling needs the overflow decision on the host
            bad = torch.tensor([0.0 if torch.isfinite(g).all() else 1.0], device=self.device)
            if self.world > 1:
                dist.all_reduce(bad, op=dist.ReduceOp.MAX)
            overflow = bad.item() > 0
            self.scaler.update(overflow)
            if overflow:
                self._skipped += 1
                self.zero_grad()
                return
        sumsq = self._global_sumsq(g) * (inv * inv)
        norm = sumsq.sqrt()
        self.last_grad_norm = norm.reshape(())
        # clip coefficient stays a device tensor: no host sync in the step (bf16 / fp32)
        if self.clip > 0:
            coef = torch.clamp(self.clip / (norm + 1e-6), max=1.0) * inv
        else:
            coef = torch.full_like(norm, inv)
        lr = self.param_groups[0]["lr"]
        self.opt_step += 1
        b1, b2 = self.betas
        if self.opt8:
            self._step_8bit(g, norm, coef, lr, b1, b2)
        elif self.offload:
            from ..ops._native import cpu_native
            gc = g.float().cpu()
            cpu_native().adamw_step(self.master, gc, self.exp_avg, self.exp_avg_sq, lr, b1, b2, self.eps, self.wd,
                                    self.opt_step, float(coef.reshape(())))
        elif use_native(self.master):
            gg = g.float().contiguous() if g.dtype != torch.float32 or not g.is_contiguous() else g
            gs = torch.cat([norm.reshape(1), coef.reshape(1)]).float()
            native().adamw(self.master, gg, self.exp_avg, self.exp_avg_sq, None, lr, b1, b2, self.eps, self.wd,
                           self.opt_step, gs, None)
        else:
            ref.adamw_step(self.master, g.float() * coef.to(g.device), self.exp_avg, self.exp_avg_sq, self.opt_step,
                           lr, b1, b2, self.eps, self.wd)
        self._publish_params()
        self.zero_grad()

    def _step_8bit(self, g, norm, coef, lr, b1, b2):
        gg = g.float().contiguous()
        if self.offload:
            gg = gg.cpu()
        if use_native(self.master):
            gs = torch.cat([norm.reshape(1), coef.reshape(1)]).float()
            native().adamw8bit(self.master, gg, self.qm, self.qv, self.am, self.av, self.code_s, self.code_u, None, lr,
                               b1, b2, self.eps, self.wd, self.opt_step, gs, None)
        else:
            from ..optim.adamw import adamw8bit_reference
            adamw8bit_reference(self.master, gg * coef.to(gg.device), self.qm, self.qv, self.am, self.av, self.code_s,
                                self.code_u, self.opt_step, lr, b1, b2, self.eps, self.wd)

    def _state_tensors(self) -> dict:
        if self.opt8:
            return {"master": self.master, "qm": self.qm, "qv": self.qv, "am": self.am, "av": self.av}
        return {"master": self.master, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}

    def _publish_params(self):
        m = self.master.to(self.device, non_blocking=True)
        if self.stage == 3:
            pers = []
            for u, o in zip(self.units, self.unit_offsets):
                u.shard.copy_(m[o:o + u.shard_n])
                if self.persistent[id(u)]:
                    pers.append(u)
                else:
                    u.release()           # stale full copies (kept for reuse / prefetched) are dropped
            if not pers:
                return
            # persistent units refresh their full copy with ONE coalesced all-gather (rank-major)
            S = sum(u.shard_n for u in pers)
            send = torch.cat([u.shard for u in pers])
            if self.world > 1:
                recv = torch.empty(self.world * S, dtype=send.dtype, device=send.device)
                dist.all_gather_into_tensor(recv, send)
                view = recv.view(self.world, S)
            else:
                view = send.view(1, S)
            col = 0
            for u in pers:
                if not u.gathered:
                    u.full.untyped_storage().resize_(u.npad * u.full.element_size())
                    u.gathered = True
                u.full.view(self.world, u.shard_n).copy_(view[:, col:col + u.shard_n])
                col += u.shard_n
            return
        self.flat_model[self.shard_slice].copy_(m)
        if self.world > 1 and self.stage > 0:
            dist.all_gather_into_tensor(self.flat_model, self.flat_model[self.shard_slice].clone())

    # ------------------------------------------------------------------ state / checkpoints
    @contextlib.contextmanager
    def gathered_params(self):
        """All stage-3 partitions gathered for the duration (collective: call on every rank);
        e.g. around an adapter ``save_pretrained`` (``stage3_gather_16bit_weights_on_model_save``)."""
        if self.stage == 3:
            for u in self.units:
                u.gather()
        try:
            yield
        finally:
            if self.stage == 3:
                for u in self.units:
                    if not self.persistent[id(u)]:
                        u.release()

    def consolidated_state_dict(self) -> dict:
        """Full (16-bit where trained in 16-bit) model state dict; gathers stage-3 shards."""
        if self.stage == 3:
            for u in self.units:
                u.gather()
        sd = {k: v.detach().clone() for k, v in self.module.state_dict().items()}
        if self.stage == 3:
            for u in self.units:
                if not self.persistent[id(u)]:
                    u.release()
        return sd

    def save_checkpoint(self, save_dir: str, tag: str | None = None, client_state: dict | None = None):
        tag = tag or f"global_step{self.global_steps}"
        d = os.path.join(save_dir, tag)
        os.makedirs(d, exist_ok=True)
        module = None
        if self.stage < 3 or self.cfg.zero.stage3_gather_16bit_weights_on_model_save:
            module = self.consolidated_state_dict()     # collective under stage 3
        if self.rank == 0:
            torch.save({"module": module, "global_steps": self.global_steps, "micro_steps": self.micro_steps,
                        "loss_scale": self.scaler.scale, "client_state": client_state or {},
                        "ds_config": self.cfg.raw, "zero_stage": self.stage, "world_size": self.world},
                       os.path.join(d, "mp_rank_00_model_states.pt"))
        torch.save({**{k: v.cpu() for k, v in self._state_tensors().items()}, "optim": self.optim_name,
                    "opt_step": self.opt_step, "zero_stage": self.stage, "rank": self.rank, "world": self.world,
                    "layout": self._layout(), "block": self.block,
                    "lr_scheduler": self.lr_scheduler.state_dict() if self.lr_scheduler else None},
                   os.path.join(d, f"zero_pp_rank_{self.rank}_mp_rank_00_optim_states.pt"))
        if is_dist():
            dist.barrier()
        if self.rank == 0:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(tag)
        return d

    def load_checkpoint(self, load_dir: str, tag: str | None = None):
        if tag is None:
            with open(os.path.join(load_dir, "latest")) as f:
                tag = f.read().strip()
        d = os.path.join(load_dir, tag)
        ms = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
        os_ = torch.load(os.path.join(d, f"zero_pp_rank_{min(self.rank, ms.get('world_size', 1) - 1)}_mp_rank_00_optim_states.pt"),
                         map_location="cpu", weights_only=True)
        if os_.get("optim", "adamw") != self.optim_name:
            raise ValueError(f"checkpoint optimizer {os_.get('optim', 'adamw')!r} != engine optimizer {self.optim_name!r}")
        st = self._state_tensors()
        if os_["world"] == self.world:
            for k, t in st.items():
                t.copy_(os_[k])
        else:                             # re-partition: rebuild the full vectors from every old shard
            old = [torch.load(os.path.join(d, f"zero_pp_rank_{r}_mp_rank_00_optim_states.pt"), map_location="cpu",
                              weights_only=True) for r in range(os_["world"])]
            ob = os_.get("block", 1)
            for k, t in st.items():
                if k in ("am", "av"):     # per-256-block scales: the same layout, counted in blocks
                    lay = [(_pad_to(max(n, 1), 256)) // 256 for n in (os_.get("layout") or self._layout())]
                    full = self._unshard([o[k] for o in old], lay, os_["world"], ob // 256 if ob >= 256 else 1)
                    t.copy_(self._shard_of(full, block_units=True))
                else:
                    full = self._unshard([o[k] for o in old], os_.get("layout"), os_["world"], ob)
                    # the 8-bit moments' padding must decode to 0: the index of the code nearest 0
                    # (code 0 of the signed dynamic map is about -1.0, a phantom moment)
                    fill = (int(torch.argmin(self.code_s.abs())) if k == "qm" else
                            int(torch.argmin(self.code_u.abs())) if k == "qv" else 0)
                    t.copy_(self._shard_of(full, fill=fill))
        self.opt_step = os_["opt_step"]
        if self.lr_scheduler is not None and os_.get("lr_scheduler"):
            self.lr_scheduler.load_state_dict(os_["lr_scheduler"])
        self.global_steps, self.micro_steps = ms["global_steps"], ms["micro_steps"]
        self.scaler.scale = ms["loss_scale"]
        self._publish_params()
        return d, ms.get("client_state", {})

    # ------------------------------------------------------------------ re-partitioning helpers
    def _layout(self) -> list[int]:
        """World-independent partition layout: numel per stage-3 unit, or [n] for stages 0-2."""
        return [u.n for u in self.units] if self.stage == 3 else [self.n]

    def _unshard(self, shards: list[torch.Tensor], layout, world_old: int, block_old: int = 1) -> torch.Tensor:
        layout = layout or self._layout()
        if self.stage == 0:               # replicated state
            return shards[0][:layout[0]]
        parts, offs = [], [0] * world_old
        for n in layout:
            sn = _pad_to(max(n, 1), world_old * block_old) // world_old
            full = torch.cat([shards[r][offs[r]:offs[r] + sn] for r in range(world_old)])
            parts.append(full[:n])
            offs = [o + sn for o in offs]
        return torch.cat(parts)

    def _shard_of(self, full: torch.Tensor, block_units: bool = False, fill: int = 0) -> torch.Tensor:
        """This rank's shard of a full (unpadded) state vector in the current layout
        (``block_units``: the vector counts 256-element blocks — the 8-bit state scales; ``fill``: the
        value of the padded tail)."""
        d = 256 if block_units else 1
        if self.stage == 3:
            out, o = [], 0
            for u in self.units:
                n = (_pad_to(max(u.n, 1), 256) // 256) if block_units else u.n
                v = torch.full((u.npad // d,), fill, dtype=full.dtype)
                v[:n] = full[o:o + n]
                sn = u.shard_n // d
                out.append(v[self.rank * sn:(self.rank + 1) * sn])
                o += n
            return torch.cat(out)
        n = (_pad_to(max(self.n, 1), 256) // 256) if block_units else self.n
        v = torch.full((self.npad // d,), fill, dtype=full.dtype)
        v[:n] = full[:n]
        sn = self.shard_n // d
        r0 = self.shard_slice.start // self.shard_n if self.shard_n else 0
        return v[r0 * sn:(r0 + 1) * sn]

    # DeepSpeed accessors used by the reference scripts
    def train_micro_batch_size_per_gpu(self):
        return self.cfg.train_micro_batch_size_per_gpu

    def gradient_accumulation_steps(self):
        return self.ga

    def get_lr(self):
        return [self.param_groups[0]["lr"]]

    def get_global_grad_norm(self):
        return float(self.last_grad_norm)

    @property
    def skipped_steps(self):
        return self._skipped


def initialize(model: nn.Module, config, model_parameters=None, optimizer=None, lr_scheduler=None, **kw):
    """``deepspeed.initialize`` analogue → (engine, optimizer, dataloader=None, lr_scheduler).

    A client ``optimizer`` is accepted for API compatibility; when the config also declares an
    ``optimizer`` block the config wins (documented precedence), otherwise the client's
    ``lr`` / ``weight_decay`` / ``betas`` / ``eps`` are adopted."""
    lr = wd = None
    betas, eps = (0.9, 0.999), 1e-8
    if optimizer is not None and hasattr(optimizer, "param_groups"):
        g = optimizer.param_groups[0]
        lr, wd = g.get("lr"), g.get("weight_decay")
        betas, eps = g.get("betas", betas), g.get("eps", eps)
    engine = ZeroEngine(model, config, lr=lr, weight_decay=wd, betas=betas, eps=eps, **kw)
    return engine, engine, None, engine.lr_scheduler
