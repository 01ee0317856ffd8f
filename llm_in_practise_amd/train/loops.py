"""Training loop for the from-scratch language models (SURVEY.md tracks A-D: MiniGPT, GPTLike,
DeepSeekLike) with the reference's parallel strategies mapped onto this framework:

===============  ===========================================================  ==========================
strategy         reference                                                    here
===============  ===========================================================  ==========================
single           ``GPTLike_wikitext2_*.py``, ``GPTLike-Bert-Wikitext2.py``    plain loop
ddp              ``ddp_basics/ddp_gpt_wikitext2.py:274``                       flat-buffer DDP over RCCL
fsdp / fsdp2     ``fsdp_basics/fsdp_gpt_wikitext2.py:278-312`` / ``fsdp2_*``  ZeRO-3 engine (per block)
zero1/2/3        ``DeepSpeed-GPTLike-ZeRO-{1,2,3}/ds_config.json``            ZeRO engine, ds_config
zero-offload     ``DeepSpeed-GPTLike-ZeRO-Offload``                            ZeRO-3 + host AdamW
===============  ===========================================================  ==========================

Checkpoints follow each family's layout: per-epoch ``{epoch, model/optimizer/scheduler state,
vocab_size, block_size, args}`` with keep-last-N rotation (``GPTLike_wikitext2_fixed_pe.py:382-401``),
rank-0 ``checkpoints/model_epoch_{n}.pth`` + ``models/final_model.pth`` (DDP/FSDP, ``ddp_gpt_wikitext2.py:322-331``),
and the DeepSpeed ``<save_dir>/epoch{n}/`` shard layout (``DeepSpeed-GPTLike-ZeRO-1.py:322-330``).
Every collective (save, eval reduce) is entered by all ranks (the reference's rank-0-only
``save_checkpoint`` deadlock, SURVEY §5.2 item 2, cannot happen here).
"""
from __future__ import annotations

import dataclasses
import math
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..optim.adamw import LRScheduler, build_optimizer, decay_param_groups
from ..parallel import dist as D
from ..utils.logging import get_logger


@dataclasses.dataclass
class LoopConfig:
    epochs: int = 3
    batch_size: int = 16
    lr: float = 3e-4
    weight_decay: float = 0.01
    clip_grad_norm: float = 1.0
    grad_accum: int = 1
    strategy: str = "single"
    ds_config: str | dict | None = None
    precision: str = "fp32"            # fp32 | bf16 | fp16
    scheduler: str = "none"            # none | step | cosine | warmup_lr
    step_per_batch: bool = False       # B2/B4/B6 step StepLR per batch (documented reference bug)
    gamma: float = 0.95
    log_every: int = 50
    save_dir: str | None = None
    save_interval: int = 1
    keep_last: int = 5
    final_model: str | None = None
    seed: int = 42
    max_steps: int = -1
    eval_every_epoch: bool = False
    # temp/ddp_gpt_bpe_tokenizer_02.py parity (C6): validation split, best model, early stop, resume
    patience: int = 0                  # epochs without val improvement before stopping (0 = off)
    best_model: str | None = None      # path for the best-validation weights (rank 0)
    resume: bool = False               # continue from <save_dir>/latest_checkpoint.pt if present
    no_decay_groups: bool = False      # temp/ddp_gpt_wikitext2.py:337-344: biases / LayerNorm without decay


def lm_loss(model: nn.Module, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    out = model(x, y) if _takes_targets(model) else model(x)
    if isinstance(out, tuple) and out[1] is not None:
        return out[1]
    logits = out[0] if isinstance(out, tuple) else out
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), y.reshape(-1))


def _takes_targets(model) -> bool:
    import inspect
    m = getattr(model, "module", model)
    try:
        return len(inspect.signature(m.forward).parameters) >= 2
    except (TypeError, ValueError):
        return False


def _sampler_indices(n, world, rank, epoch, seed, shuffle=True):
    g = torch.Generator().manual_seed(seed + epoch)
    idx = torch.randperm(n, generator=g).tolist() if shuffle else list(range(n))
    per = math.ceil(n / world)
    idx = (idx + idx[:per * world - n])[rank::world]
    return idx


def _batches(ds, idx, bs):
    for s in range(0, len(idx) - bs + 1, bs):
        rows = [ds[j] for j in idx[s:s + bs]]
        yield torch.stack([torch.as_tensor(r[0]) for r in rows]), torch.stack([torch.as_tensor(r[1]) for r in rows])


def _ds_config_for(strategy: str, cfg: LoopConfig) -> dict:
    if cfg.ds_config is not None:
        return cfg.ds_config
    stage = {"zero1": 1, "zero2": 2, "zero3": 3, "zero-offload": 3, "fsdp": 3, "fsdp2": 3}[strategy]
    d = {"train_micro_batch_size_per_gpu": cfg.batch_size, "gradient_accumulation_steps": cfg.grad_accum,
         "gradient_clipping": cfg.clip_grad_norm,
         "optimizer": {"type": "AdamW", "params": {"lr": cfg.lr, "weight_decay": cfg.weight_decay}},
         "zero_optimization": {"stage": stage, "stage3_param_persistence_threshold": 0}}
    if strategy == "zero-offload":
        d["zero_optimization"]["offload_optimizer"] = {"device": "cpu", "pin_memory": torch.cuda.is_available()}
    if cfg.precision == "bf16":
        d["bf16"] = {"enabled": True}
    elif cfg.precision == "fp16":
        d["fp16"] = {"enabled": True, "loss_scale": 0, "initial_scale_power": 16}
    return d


def train_lm(model: nn.Module, train_ds, cfg: LoopConfig, eval_ds=None, meta: dict | None = None) -> dict:
    log = get_logger("lipa.loop")
    world, rank = D.world_size(), D.rank()
    dev = next(model.parameters()).device
    torch.manual_seed(cfg.seed)
    engine = ddp = None
    if cfg.strategy in ("zero1", "zero2", "zero3", "zero-offload", "fsdp", "fsdp2"):
        from ..parallel.zero import ZeroEngine
        engine = ZeroEngine(model, _ds_config_for(cfg.strategy, cfg), lr=cfg.lr, weight_decay=cfg.weight_decay,
                            micro_batch=cfg.batch_size, grad_accum=cfg.grad_accum)
        opt = engine
        bs = engine.train_micro_batch_size_per_gpu() or cfg.batch_size   # ds_config overrides --batch_size
    else:
        if cfg.precision == "bf16":
            model.to(torch.bfloat16)
        params = (decay_param_groups(model, cfg.weight_decay) if cfg.no_decay_groups
                  else [p for p in model.parameters() if p.requires_grad])
        opt = build_optimizer("adamw", params, cfg.lr, cfg.weight_decay, max_grad_norm=cfg.clip_grad_norm)
        if cfg.strategy == "ddp" and world > 1:
            from ..parallel.ddp import DistributedDataParallel
            ddp = DistributedDataParallel(model, flat=opt.flat)
        bs = cfg.batch_size
    n = len(train_ds)
    steps_per_epoch = max(1, (math.ceil(n / world) // bs) // cfg.grad_accum)
    total = cfg.max_steps if cfg.max_steps > 0 else steps_per_epoch * cfg.epochs
    sched = None
    if cfg.scheduler == "step":
        sched = LRScheduler(opt, "step", cfg.lr, total, gamma=cfg.gamma,
                            step_size=1 if cfg.step_per_batch else steps_per_epoch)
    elif cfg.scheduler == "cosine":
        sched = LRScheduler(opt, "cosine", cfg.lr, total)
    elif engine is not None and engine.lr_scheduler is not None:
        sched = None                         # engine steps its own (ds_config WarmupLR)
    hist = {"train_loss": [], "eval_loss": [], "step_time": []}
    step = 0
    start_epoch, best, bad = 0, float("inf"), 0
    latest = os.path.join(cfg.save_dir, "latest_checkpoint.pt") if cfg.save_dir else None
    if cfg.resume and engine is None and latest and os.path.exists(latest):
        st = _load_latest(latest, model, opt, sched, dev)
        start_epoch, step, best, bad = st["epoch"], st["global_step"], st["best_val_loss"], st["bad_epochs"]
        hist = st.get("history", hist)
        if rank == 0:
            log.info(f"resumed from {latest}: epoch {start_epoch}, step {step}")
    from ..utils.faults import FaultInjector
    faults = FaultInjector()                   # FAULT_INJECT=rank:step:kind (resume / failure tests)
    for epoch in range(start_epoch, cfg.epochs):
        model.train()
        idx = _sampler_indices(n, world, rank, epoch, cfg.seed)
        tot, cnt, t0 = 0.0, 0, time.time()
        for bi, (x, y) in enumerate(_batches(train_ds, idx, bs)):
            x, y = x.to(dev), y.to(dev)
            boundary = (bi + 1) % cfg.grad_accum == 0
            if engine is not None:
                loss = lm_loss(engine.module, x, y)
                engine.backward(loss)
                engine.step()
            else:
                ctx = ddp.no_sync() if (ddp is not None and not boundary) else _Null()
                with ctx:
                    loss = lm_loss(model, x, y)
                    (loss / cfg.grad_accum).backward()
                if boundary:
                    if hasattr(opt, "flat"):
                        opt.flat.sync_grads()
                    if ddp is not None:
                        ddp.allreduce_grads()
                    if cfg.clip_grad_norm > 0:
                        opt.clip_grad_norm_(cfg.clip_grad_norm)
                    opt.step()
                    opt.zero_grad()
            if boundary:
                step += 1
                if sched is not None:
                    sched.step()
                if faults:
                    faults.check(step)
            tot += float(loss.detach())
            cnt += 1
            if rank == 0 and cfg.log_every and (bi + 1) % cfg.log_every == 0:
                log.info(f"epoch {epoch + 1} batch {bi + 1} loss {tot / cnt:.4f}")
            if 0 < cfg.max_steps <= step:
                break
        avg = tot / max(1, cnt)
        if world > 1:
            t = torch.tensor([avg], device=dev)
            D.all_reduce_mean_(t)
            avg = float(t)
        hist["train_loss"].append(avg)
        hist["step_time"].append((time.time() - t0) / max(1, cnt))
        stop = False
        if eval_ds is not None and cfg.eval_every_epoch:
            val = evaluate_lm(engine.module if engine else model, eval_ds, bs)   # identical on every rank
            hist["eval_loss"].append(val)
            if val < best:
                best, bad = val, 0
                if cfg.best_model:
                    sd = engine.consolidated_state_dict() if engine is not None else model.state_dict()
                    if rank == 0:
                        os.makedirs(os.path.dirname(cfg.best_model) or ".", exist_ok=True)
                        torch.save({"epoch": epoch + 1, "val_loss": val, "model_state_dict": sd, **(meta or {})},
                                   cfg.best_model)
            else:
                bad += 1
                stop = cfg.patience > 0 and bad >= cfg.patience
        if rank == 0:
            log.info(f"epoch {epoch + 1}/{cfg.epochs} train loss {avg:.4f}"
                     + (f" val loss {hist['eval_loss'][-1]:.4f}" if hist["eval_loss"] else ""))
        if cfg.save_dir and (epoch + 1) % cfg.save_interval == 0:
            save_epoch_checkpoint(model, opt, sched, engine, cfg, epoch + 1, meta or {})
        if latest and engine is None:
            _save_latest(latest, model, opt, sched, epoch + 1, step, best, bad, hist)
        if stop:
            if rank == 0:
                log.info(f"early stop: no val improvement for {cfg.patience} epochs")
            break
        if 0 < cfg.max_steps <= step:
            break
    hist["global_step"] = step
    if cfg.final_model:
        sd = engine.consolidated_state_dict() if engine is not None else model.state_dict()
        if rank == 0:
            os.makedirs(os.path.dirname(cfg.final_model) or ".", exist_ok=True)
            torch.save(sd, cfg.final_model)
    return hist


@torch.no_grad()
def evaluate_lm(model, ds, bs: int = 16) -> float:
    """Distributed mean loss (the reference's ``dist.reduce`` ×2 + broadcast,
    ``temp/ddp_gpt_bpe_tokenizer_02.py:305-345``, as one all-reduce of [sum, count])."""
    model.eval()
    dev = next(model.parameters()).device
    idx = _sampler_indices(len(ds), D.world_size(), D.rank(), 0, 0, shuffle=False)
    acc = torch.zeros(2, device=dev, dtype=torch.float64)
    for x, y in _batches(ds, idx, bs):
        loss = lm_loss(model, x.to(dev), y.to(dev))
        acc[0] += float(loss) * x.shape[0]
        acc[1] += x.shape[0]
    if D.is_dist():
        import torch.distributed as dist
        dist.all_reduce(acc)
    model.train()
    return float(acc[0] / acc[1].clamp(min=1))


def save_epoch_checkpoint(model, opt, sched, engine, cfg: LoopConfig, epoch: int, meta: dict):
    if engine is not None:                       # collective: every rank
        engine.save_checkpoint(cfg.save_dir, tag=f"epoch{epoch}")
        return
    if D.rank() != 0:
        return
    os.makedirs(cfg.save_dir, exist_ok=True)
    path = os.path.join(cfg.save_dir, f"model_epoch_{epoch}.pth")
    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(),
                "optimizer_state_dict": opt.state_dict(),
                "scheduler_state_dict": sched.state_dict() if sched is not None else None,
                "args": {k: v for k, v in dataclasses.asdict(cfg).items() if not isinstance(v, dict)}, **meta}, path)
    if cfg.keep_last:
        old = os.path.join(cfg.save_dir, f"model_epoch_{epoch - cfg.keep_last}.pth")
        if os.path.exists(old):
            os.remove(old)


def _rng_state() -> dict:
    import random
    import numpy as np
    st = {"python": random.getstate(), "numpy": np.random.get_state(), "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st: dict):
    import random
    import numpy as np
    random.setstate(st["python"])
    np.random.set_state(st["numpy"])
    torch.set_rng_state(st["torch"])
    if torch.cuda.is_available() and "cuda" in st:
        torch.cuda.set_rng_state_all(st["cuda"])


def _save_latest(path, model, opt, sched, epoch, step, best, bad, hist):
    """``latest_checkpoint.pt`` with everything a bit-exact continuation needs (rank 0 writes;
    every rank has identical replicated state under DDP)."""
    if D.rank() != 0:
        return
    tmp = path + ".tmp"
    torch.save({"epoch": epoch, "global_step": step, "model_state_dict": model.state_dict(),
                "optimizer_state_dict": opt.state_dict(),
                "scheduler_state_dict": sched.state_dict() if sched is not None else None,
                "best_val_loss": best, "bad_epochs": bad, "history": hist, "rng": _rng_state()}, tmp)
    os.replace(tmp, path)


def _load_latest(path, model, opt, sched, dev) -> dict:
    # our own file (written by _save_latest): RNG states are Python objects, so full unpickling
    st = torch.load(path, map_location=dev, weights_only=False)
    model.load_state_dict(st["model_state_dict"])
    opt.load_state_dict(st["optimizer_state_dict"])
    if sched is not None and st["scheduler_state_dict"] is not None:
        sched.load_state_dict(st["scheduler_state_dict"])
    rng = st["rng"]
    if isinstance(rng.get("torch"), torch.Tensor):
        rng["torch"] = rng["torch"].cpu()
    if "cuda" in rng:
        rng["cuda"] = [t.cpu() for t in rng["cuda"]]
    _set_rng_state(rng)
    return st


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
