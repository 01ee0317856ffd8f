"""HF-``Trainer``-compatible training loop.

What the reference's fine-tuning scripts rely on (``Fine-Tuning/qwen3-8b-qlora-dist.py:133-175``,
``qwen3-8b-lora.py:158-204``) and what this reproduces:

* ``TrainingArguments`` with the same names (subset actually used by the reference plus a
  few MI355X knobs: ``ga_fusion``, ``metrics_jsonl``, ``wall_clock_breakdown``).
* Strategy selection like HF: ``deepspeed=<ds_config>`` → our ZeRO engine
  (``parallel/zero.py``); else world>1 → flat-buffer DDP over RCCL; else single device.
* Gradient accumulation with comm only at the boundary; optional fused-GA pass (all GA
  micro-batches in one forward/backward with per-micro-batch loss normalisation, gradient-
  identical to sequential accumulation) when the model supports ``num_micro_batches``.
* HF defaults: linear schedule without warmup, ``max_grad_norm=1.0``, ``seed=42``.
* ``checkpoint-{step}/`` = adapter (``adapter_model.safetensors`` + ``adapter_config.json``)
  or ``model.safetensors``, ``optimizer.pt``, ``scheduler.pt``, ``rng_state[_{rank}].pth``,
  ``trainer_state.json``, ``training_args.bin`` (a plain dict, loadable with
  ``weights_only=True``); rotated by ``save_total_limit``.  ZeRO runs add ``global_step{N}/``.
* Exact resume: model/optimizer/scheduler/RNG/step restored, the epoch's deterministic
  sample order is replayed and already-consumed batches skipped.
* Logging in the Trainer's console format ``{'loss': …, 'grad_norm': …, 'learning_rate': …,
  'epoch': …}`` every ``logging_steps`` plus a JSONL metrics stream; ``log_metrics`` /
  ``save_metrics("train")`` → ``train_results.json`` / ``all_results.json``.
* ``FAULT_INJECT`` hook (``utils/faults.py``) for resume / failure tests.
"""
from __future__ import annotations

import dataclasses
import glob
import inspect
import json
import math
import os
import random
import re
import shutil
import time

import numpy as np
import torch
import torch.nn as nn

from ..optim.adamw import LRScheduler, build_optimizer
from ..parallel import dist as D
from ..utils.faults import FaultInjector
from ..utils.gc_control import ManualGC
from ..utils.logging import get_logger
from ..utils.metrics import MetricsWriter
from ..utils.timer import StepTimer

PREFIX_CHECKPOINT_DIR = "checkpoint"


@dataclasses.dataclass
class TrainingArguments:
    output_dir: str = "./output"
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    num_train_epochs: float = 3.0
    max_steps: int = -1
    learning_rate: float = 5e-5
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    max_grad_norm: float = 1.0
    lr_scheduler_type: str = "linear"
    warmup_steps: int = 0
    warmup_ratio: float = 0.0
    logging_steps: int = 10
    logging_dir: str | None = None
    save_strategy: str = "steps"
    save_steps: int = 500
    save_total_limit: int | None = None
    bf16: bool = False
    fp16: bool = False
    gradient_checkpointing: bool = False
    gradient_checkpointing_kwargs: dict | None = None
    optim: str = "adamw_torch"
    seed: int = 42
    report_to: list | str | None = None
    remove_unused_columns: bool = True
    ddp_backend: str | None = None
    ddp_timeout: int = 1800
    ddp_find_unused_parameters: bool | None = None
    deepspeed: str | dict | None = None
    dataloader_num_workers: int = 0
    dataloader_drop_last: bool = False
    eval_strategy: str = "no"
    eval_steps: int | None = None
    load_best_model_at_end: bool = False
    metric_for_best_model: str | None = None
    greater_is_better: bool | None = None
    resume_from_checkpoint: str | None = None
    local_rank: int = -1
    # MI355X-native additions
    ga_fusion: bool = True
    metrics_jsonl: str | None = None
    wall_clock_breakdown: bool = False

    def to_dict(self):
        return dataclasses.asdict(self)


@dataclasses.dataclass
class TrainerState:
    global_step: int = 0
    epoch: float = 0.0
    max_steps: int = 0
    num_train_epochs: int = 0
    logging_steps: int = 10
    save_steps: int = 500
    total_flos: float = 0.0
    log_history: list = dataclasses.field(default_factory=list)
    best_metric: float | None = None
    best_model_checkpoint: str | None = None
    train_batch_size: int = 0

    def save_to_json(self, path):
        with open(path, "w") as f:
            json.dump(dataclasses.asdict(self), f, indent=2)

    @classmethod
    def load_from_json(cls, path):
        with open(path) as f:
            d = json.load(f)
        return cls(**{k: v for k, v in d.items() if k in {f.name for f in dataclasses.fields(cls)}})


class EvalPrediction(tuple):
    """``(predictions, label_ids)`` as handed to ``compute_metrics``."""

    def __new__(cls, predictions, label_ids):
        return super().__new__(cls, (predictions, label_ids))

    @property
    def predictions(self):
        return self[0]

    @property
    def label_ids(self):
        return self[1]


@dataclasses.dataclass
class TrainOutput:
    global_step: int
    training_loss: float
    metrics: dict


def set_seed(seed: int):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    from ..ops.linear import seed_dropout
    seed_dropout(seed)


def _rng_state():
    from ..ops.linear import _KEY
    st = {"python": random.getstate(), "numpy": np.random.get_state(), "cpu": torch.get_rng_state(),
          "dropout_key": int(_KEY[0])}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st):
    random.setstate(st["python"])
    np.random.set_state(st["numpy"])
    torch.set_rng_state(st["cpu"])
    if "dropout_key" in st:
        from ..ops.linear import _KEY
        _KEY[0] = int(st["dropout_key"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["cuda"])


def _rng_to_safe(st):
    """RNG state as tensors / plain containers so it reloads with ``weights_only=True``."""
    py = st["python"]
    npst = st["numpy"]
    out = {"python": [py[0], list(py[1]), py[2]],
           "numpy": [npst[0], torch.from_numpy(np.asarray(npst[1]).astype(np.int64)), int(npst[2]), int(npst[3]),
                     float(npst[4])],
           "cpu": st["cpu"], "dropout_key": st.get("dropout_key", 0)}
    if "cuda" in st:
        out["cuda"] = list(st["cuda"])
    return out


def _rng_from_safe(d):
    py = d["python"]
    npst = d["numpy"]
    st = {"python": (py[0], tuple(py[1]), py[2]),
          "numpy": (npst[0], npst[1].numpy().astype(np.uint32), npst[2], npst[3], npst[4]),
          "cpu": d["cpu"], "dropout_key": d.get("dropout_key", 0)}
    if "cuda" in d:
        st["cuda"] = d["cuda"]
    return st


class _EpochSampler:
    """Deterministic per-epoch shuffle (seed + epoch), rank-strided shards (DistributedSampler
    semantics: padded by wrap-around so every rank gets the same count)."""

    def __init__(self, n, world, rank, seed, shuffle=True, drop_last=False):
        self.n, self.world, self.rank, self.seed, self.shuffle = n, world, rank, seed, shuffle
        self.num = n // world if drop_last else math.ceil(n / world)

    def indices(self, epoch):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        total = self.num * self.world
        idx = (idx + idx[:total - len(idx)]) if total > len(idx) else idx[:total]
        return idx[self.rank:total:self.world]


def default_collate(rows):
    if isinstance(rows[0], dict):
        out = {}
        for k in rows[0]:
            v = [r[k] for r in rows]
            out[k] = torch.stack([torch.as_tensor(x) for x in v])
        return out
    if isinstance(rows[0], (tuple, list)):
        return type(rows[0])(torch.stack([torch.as_tensor(r[i]) for r in rows]) for i in range(len(rows[0])))
    return torch.stack([torch.as_tensor(r) for r in rows])


def _unwrap(m):
    while hasattr(m, "module") and isinstance(getattr(m, "module"), nn.Module):
        m = m.module
    return m


class Trainer:
    def __init__(self, model: nn.Module, args: TrainingArguments, train_dataset=None, eval_dataset=None,
                 data_collator=None, tokenizer=None, processing_class=None, optimizers=(None, None),
                 compute_loss_fn=None, callbacks=None, compute_metrics=None):
        self.args = args
        self.model = model
        self.train_dataset, self.eval_dataset = train_dataset, eval_dataset
        self.data_collator = data_collator or default_collate
        self.tokenizer = processing_class or tokenizer
        self.optimizer, self.lr_scheduler = optimizers
        self.compute_loss_fn = compute_loss_fn
        self.compute_metrics = compute_metrics
        self.callbacks = callbacks or []
        self.state = TrainerState(logging_steps=args.logging_steps, save_steps=args.save_steps)
        if os.environ.get("WORLD_SIZE") and int(os.environ["WORLD_SIZE"]) > 1 and not D.is_dist():
            D.init_distributed(backend=args.ddp_backend, timeout_s=args.ddp_timeout)
        self.world, self.rank = D.world_size(), D.rank()
        self.device = next(model.parameters()).device
        self.log = get_logger("lipa.trainer", os.path.join(args.logging_dir, "training.log") if args.logging_dir
                              else None)
        self.metrics = MetricsWriter(args.metrics_jsonl, self.rank)
        self.timer = StepTimer(args.wall_clock_breakdown)
        self.faults = FaultInjector()
        self.engine = None
        self.ddp = None
        self._interrupt_dir = None
        if args.gradient_checkpointing and hasattr(_unwrap(model), "gradient_checkpointing_enable"):
            _unwrap(model).gradient_checkpointing_enable(args.gradient_checkpointing_kwargs)

    # ------------------------------------------------------------------ helpers
    def is_world_process_zero(self):
        return self.rank == 0

    def _trainable(self):
        return [p for p in self.model.parameters() if p.requires_grad]

    def _model_accepts(self, name):
        try:
            return name in inspect.signature(_unwrap(self.model).forward).parameters or \
                name in inspect.signature(getattr(_unwrap(self.model), "model", _unwrap(self.model)).forward).parameters
        except (TypeError, ValueError):
            return False

    def _total_steps(self, steps_per_epoch):
        if self.args.max_steps > 0:
            return self.args.max_steps
        return max(1, math.ceil(self.args.num_train_epochs * steps_per_epoch))

    def create_optimizer_and_scheduler(self, total_steps):
        a = self.args
        if a.deepspeed:
            from ..parallel.zero import ZeroEngine
            hidden = getattr(getattr(_unwrap(self.model), "config", None), "hidden_size", None)
            self.engine = ZeroEngine(self.model, a.deepspeed, lr=a.learning_rate, weight_decay=a.weight_decay,
                                     betas=(a.adam_beta1, a.adam_beta2), eps=a.adam_epsilon, hidden_size=hidden,
                                     micro_batch=a.per_device_train_batch_size,
                                     grad_accum=a.gradient_accumulation_steps, total_steps=total_steps,
                                     optim=a.optim)     # client optimizer (paged_adamw_8bit) under ZeRO
            if self.engine.cfg.gradient_clipping == 0 and a.max_grad_norm > 0:
                self.engine.clip = a.max_grad_norm
            self.optimizer = self.engine
        if self.optimizer is None:
            self.optimizer = build_optimizer(a.optim, self._trainable(), a.learning_rate, a.weight_decay,
                                             (a.adam_beta1, a.adam_beta2), a.adam_epsilon, a.max_grad_norm)
        if self.lr_scheduler is None:
            if self.engine is not None and self.engine.lr_scheduler is not None:
                self.lr_scheduler = self.engine.lr_scheduler
            else:
                warm = a.warmup_steps or int(a.warmup_ratio * total_steps)
                kind = {"linear": "linear", "cosine": "cosine", "constant": "constant",
                        "constant_with_warmup": "constant"}.get(a.lr_scheduler_type, a.lr_scheduler_type)
                self.lr_scheduler = LRScheduler(self.optimizer, kind, a.learning_rate, total_steps, warm)
        if self.engine is None and self.world > 1:
            from ..parallel.ddp import DistributedDataParallel
            gb = getattr(self.optimizer, "grad_buffer", None)
            self.ddp = DistributedDataParallel(self.model, grad_buffer=gb if isinstance(gb, torch.Tensor) else None,
                                               flat=getattr(self.optimizer, "flat", None))

    # ------------------------------------------------------------------ loss
    def _to_device(self, batch):
        if isinstance(batch, dict):
            return {k: (v.to(self.device, non_blocking=True) if isinstance(v, torch.Tensor) else v)
                    for k, v in batch.items()}
        if isinstance(batch, (tuple, list)):
            return type(batch)(v.to(self.device, non_blocking=True) for v in batch)
        return batch.to(self.device)

    def compute_loss(self, model, inputs, num_micro_batches=1):
        if self.compute_loss_fn is not None:
            return self.compute_loss_fn(model, inputs)
        if isinstance(inputs, dict):
            kw = dict(inputs)
            if num_micro_batches > 1:
                kw["num_micro_batches"] = num_micro_batches
            out = model(**kw)
            return out.loss if hasattr(out, "loss") else out["loss"] if isinstance(out, dict) else out[1]
        x, y = inputs
        out = model(x, y)
        return out[1] if isinstance(out, tuple) else out

    @staticmethod
    def _count_tokens(batch):
        if isinstance(batch, dict) and "input_ids" in batch:
            ids = batch["input_ids"]
            am = batch.get("attention_mask")
            return ids.numel(), int(am.sum()) if am is not None else ids.numel()
        x = batch[0] if isinstance(batch, (tuple, list)) else batch
        return x.numel(), x.numel()

    # ------------------------------------------------------------------ checkpoint
    def _save_weights(self, out):
        m = _unwrap(self.model)
        gather = self.engine.gathered_params() if self.engine is not None else _null()
        with gather:                                  # collective under ZeRO-3: every rank enters
            if self.rank != 0:
                return
            os.makedirs(out, exist_ok=True)
            if hasattr(m, "save_pretrained") and hasattr(m, "adapter_state_dict"):
                m.save_pretrained(out)
            else:
                from safetensors.torch import save_file
                seen, clean = set(), {}
                for k, v in m.state_dict().items():   # safetensors rejects shared storage (tied heads)
                    key = (v.data_ptr(), tuple(v.shape))
                    if key in seen:
                        continue
                    seen.add(key)
                    clean[k] = v.detach().contiguous().cpu()
                save_file(clean, os.path.join(out, "model.safetensors"), metadata={"format": "pt"})
            if self.tokenizer is not None and hasattr(self.tokenizer, "save_pretrained"):
                self.tokenizer.save_pretrained(out)

    def save_model(self, output_dir: str | None = None):
        self._save_weights(output_dir or self.args.output_dir)

    def _save_checkpoint(self):
        a = self.args
        ck = os.path.join(a.output_dir, f"{PREFIX_CHECKPOINT_DIR}-{self.state.global_step}")
        self._save_weights(ck)
        if self.engine is not None:
            self.engine.save_checkpoint(ck, tag=f"global_step{self.state.global_step}")
        elif self.rank == 0:
            torch.save(self.optimizer.state_dict(), os.path.join(ck, "optimizer.pt"))
        if self.rank == 0:
            if self.lr_scheduler is not None:
                torch.save(self.lr_scheduler.state_dict(), os.path.join(ck, "scheduler.pt"))
            self.state.save_to_json(os.path.join(ck, "trainer_state.json"))
            torch.save(self.args.to_dict(), os.path.join(ck, "training_args.bin"))
        os.makedirs(ck, exist_ok=True)
        name = f"rng_state_{self.rank}.pth" if self.world > 1 else "rng_state.pth"
        torch.save(_rng_to_safe(_rng_state()), os.path.join(ck, name))
        D.barrier()
        if self.rank == 0:
            self._rotate_checkpoints()
        return ck

    def _sorted_checkpoints(self):
        cks = glob.glob(os.path.join(self.args.output_dir, f"{PREFIX_CHECKPOINT_DIR}-*"))
        cks = [c for c in cks if re.search(r"-(\d+)$", c)]
        return sorted(cks, key=lambda c: int(re.search(r"-(\d+)$", c).group(1)))

    def _rotate_checkpoints(self):
        lim = self.args.save_total_limit
        if not lim or lim <= 0:
            return
        cks = self._sorted_checkpoints()
        best = self.state.best_model_checkpoint
        if best in cks and len(cks) > lim:         # HF keeps the best checkpoint out of the rotation
            cks.remove(best)
            lim -= 1
        for c in cks[:max(0, len(cks) - lim)]:
            shutil.rmtree(c, ignore_errors=True)

    def _load_checkpoint(self, ck):
        m = _unwrap(self.model)
        if os.path.exists(os.path.join(ck, "adapter_model.safetensors")) and hasattr(m, "load_adapter"):
            m.load_adapter(ck)
        elif os.path.exists(os.path.join(ck, "model.safetensors")) and self.engine is None:
            from safetensors.torch import load_file
            sd = load_file(os.path.join(ck, "model.safetensors"))
            m.load_state_dict(sd, strict=False)
        if self.engine is not None:
            self.engine.load_checkpoint(ck)
        else:
            self.optimizer.load_state_dict(torch.load(os.path.join(ck, "optimizer.pt"), map_location="cpu",
                                                      weights_only=True))
            sync = getattr(self.optimizer, "sync_params_from_master", None)
            if sync:
                sync()
        if self.lr_scheduler is not None and os.path.exists(os.path.join(ck, "scheduler.pt")):
            self.lr_scheduler.load_state_dict(torch.load(os.path.join(ck, "scheduler.pt"), weights_only=True))
        self.state = TrainerState.load_from_json(os.path.join(ck, "trainer_state.json"))
        name = f"rng_state_{self.rank}.pth" if self.world > 1 else "rng_state.pth"
        p = os.path.join(ck, name)
        if os.path.exists(p):
            _set_rng_state(_rng_from_safe(torch.load(p, weights_only=True)))

    # ------------------------------------------------------------------ train
    def get_train_batches(self, epoch, skip=0):
        bs = self.args.per_device_train_batch_size
        idx = self.sampler.indices(epoch)
        n = len(idx) // bs * bs if self.args.dataloader_drop_last else len(idx)
        for i, s in enumerate(range(0, n, bs)):
            if i < skip:
                continue
            yield self.data_collator([self.train_dataset[j] for j in idx[s:s + bs]])

    def _micro_step(self, batches, fused):
        with self.timer.phase("fwd_bwd"):
            if fused:
                cat = {k: torch.cat([b[k] for b in batches]) for k in batches[0]}
                loss = self.compute_loss(self.model, cat, num_micro_batches=len(batches))
                # drop the previous step's spent autograd graph while this forward is queued on the
                # GPU (freed at return, its teardown stalled the launch queue before the optimizer)
                self._spent_graph = None
                poison = self.faults.check(self.state.global_step + 1) if self.faults else None
                if poison == "nan":
                    loss = loss * float("nan")
                if self.engine is not None:
                    self.engine.ga = 1
                    self.engine.backward(loss)
                else:
                    loss.backward()
                self._spent_graph = loss
                return loss.detach()
            total = 0.0
            for i, b in enumerate(batches):
                last = i == len(batches) - 1
                loss = self.compute_loss(self.model, b)
                if i == 0:
                    self._spent_graph = None   # previous step's last graph, torn down under this forward
                if self.engine is not None:
                    self.engine.backward(loss)
                    if not last:
                        self.engine.step()
                else:
                    ctx = self.ddp.no_sync() if (self.ddp is not None and not last) else _null()
                    with ctx:
                        (loss / len(batches)).backward()
                total = total + loss.detach() / len(batches)
            self._spent_graph = loss
            poison = self.faults.check(self.state.global_step + 1) if self.faults else None
            if poison == "nan":
                total = total * float("nan")
            return total

    def _optimizer_step(self):
        a = self.args
        if self.engine is not None:
            with self.timer.phase("optim"):
                self.engine.step()
                if self.lr_scheduler is not None and self.lr_scheduler is not self.engine.lr_scheduler:
                    self.lr_scheduler.step()
            return self.engine.last_grad_norm
        with self.timer.phase("comm"):
            if self.ddp is not None:
                self.ddp.allreduce_grads()
        with self.timer.phase("optim"):
            gn = None
            if a.max_grad_norm and a.max_grad_norm > 0:
                if hasattr(self.optimizer, "clip_grad_norm_"):
                    gn = self.optimizer.clip_grad_norm_(a.max_grad_norm)
                else:
                    gn = torch.nn.utils.clip_grad_norm_(self._trainable(), a.max_grad_norm)
            self.optimizer.step()
            self.lr_scheduler.step()
            self.optimizer.zero_grad()
        return gn

    def train(self, resume_from_checkpoint: str | bool | None = None):
        a = self.args
        resume_from_checkpoint = resume_from_checkpoint or a.resume_from_checkpoint
        set_seed(a.seed)
        self.model.train()
        n = len(self.train_dataset)
        self.sampler = _EpochSampler(n, self.world, self.rank, a.seed, shuffle=True, drop_last=a.dataloader_drop_last)
        bs, ga = a.per_device_train_batch_size, a.gradient_accumulation_steps
        batches_per_epoch = math.ceil(self.sampler.num / bs) if not a.dataloader_drop_last else self.sampler.num // bs
        steps_per_epoch = max(1, batches_per_epoch // ga)
        total = self._total_steps(steps_per_epoch)
        self.create_optimizer_and_scheduler(total)
        self.state.max_steps = total
        self.state.num_train_epochs = math.ceil(total / steps_per_epoch)
        self.state.train_batch_size = bs
        if resume_from_checkpoint:
            ck = resume_from_checkpoint
            if ck is True:
                cks = self._sorted_checkpoints()
                ck = cks[-1] if cks else None
            if ck:
                self._load_checkpoint(ck)
                self.log.info(f"resumed from {ck} at step {self.state.global_step}")
        fused = (a.ga_fusion and ga > 1 and self.engine is None and self._model_accepts("num_micro_batches"))
        start_epoch = self.state.global_step // steps_per_epoch
        skip_batches = (self.state.global_step % steps_per_epoch) * ga
        tr_loss_sum, tr_loss_n = 0.0, 0
        log_loss, log_n = torch.zeros((), device=self.device), 0
        t_log, tok_log, tok_real_log = time.perf_counter(), 0, 0
        step_t0 = time.perf_counter()
        if self.rank == 0:
            t, al = (getattr(_unwrap(self.model), "get_nb_trainable_parameters", lambda: (None, None)))()
            self.log.info(f"***** Running training ***** examples={n} epochs={self.state.num_train_epochs} "
                          f"micro={bs} GA={ga} world={self.world} total_steps={total} fused_ga={fused} "
                          f"strategy={'zero' + str(self.engine.stage) if self.engine else 'ddp' if self.ddp else 'single'}")
        gcm = ManualGC().__enter__()   # automatic Python GC off; a full pass every LIPA_GC_INTERVAL steps
        try:
            for epoch in range(start_epoch, self.state.num_train_epochs):
                it = self.get_train_batches(epoch, skip=skip_batches if epoch == start_epoch else 0)
                while self.state.global_step < total:
                    group = []
                    for _ in range(ga):
                        b = next(it, None)
                        if b is None:
                            break
                        group.append(self._to_device(b))
                    if len(group) < ga:
                        break                       # HF drops an incomplete trailing GA group
                    loss = self._micro_step(group, fused and all(isinstance(b, dict) for b in group)
                                            and len({tuple(b["input_ids"].shape) for b in group}) == 1)
                    gn = self._optimizer_step()
                    gcm.step()
                    self.state.global_step += 1
                    self.state.epoch = epoch + (self.state.global_step - epoch * steps_per_epoch) / steps_per_epoch
                    log_loss = log_loss + loss
                    log_n += 1
                    for b in group:
                        t_, r_ = self._count_tokens(b)
                        tok_log += t_
                        tok_real_log += r_
                    if self.state.global_step % a.logging_steps == 0 or self.state.global_step == total:
                        self._log_step(log_loss, log_n, gn, t_log, tok_log, tok_real_log)
                        tr_loss_sum += float(log_loss)
                        tr_loss_n += log_n
                        log_loss, log_n = torch.zeros((), device=self.device), 0
                        t_log, tok_log, tok_real_log = time.perf_counter(), 0, 0
                    if a.save_strategy == "steps" and a.save_steps and self.state.global_step % a.save_steps == 0:
                        self._save_checkpoint()
                    for cb in self.callbacks:
                        cb(self)
                if a.eval_strategy == "epoch" and self.eval_dataset is not None:
                    self._eval_and_track()
                if a.save_strategy == "epoch":
                    self._save_checkpoint()
                    self._track_best()
                if self.state.global_step >= total:
                    break
        except BaseException:
            self._interrupt_dir = a.output_dir.rstrip("/") + "_interrupted"
            raise
        finally:
            gcm.__exit__(None, None, None)
        if log_n:
            tr_loss_sum += float(log_loss)
            tr_loss_n += log_n
        self._spent_graph = None
        if a.load_best_model_at_end and self.state.best_model_checkpoint:
            self._load_weights_only(self.state.best_model_checkpoint)
        runtime = time.perf_counter() - step_t0
        train_loss = tr_loss_sum / max(1, tr_loss_n)
        metrics = {"train_runtime": round(runtime, 4),
                   "train_samples_per_second": round(self.state.global_step * bs * ga * self.world / runtime, 3),
                   "train_steps_per_second": round(self.state.global_step / runtime, 3),
                   "train_loss": train_loss, "epoch": self.state.epoch}
        self.state.log_history.append(dict(metrics, step=self.state.global_step))
        self.metrics.close()
        return TrainOutput(self.state.global_step, train_loss, metrics)

    def _log_step(self, log_loss, log_n, gn, t_log, tok, tok_real):
        loss = float(log_loss) / max(1, log_n)
        if self.world > 1:
            t = torch.tensor([loss], device=self.device)
            D.all_reduce_mean_(t)
            loss = float(t)
        dt = time.perf_counter() - t_log
        rec = {"loss": round(loss, 4), "grad_norm": float(gn) if gn is not None else None,
               "learning_rate": self.lr_scheduler.get_last_lr()[0] if self.lr_scheduler else None,
               "epoch": round(self.state.epoch, 4)}
        self.state.log_history.append(dict(rec, step=self.state.global_step))
        if self.rank == 0:
            print(rec, flush=True)
        extra = {"tokens_per_s": tok * self.world / dt, "nonpad_tokens_per_s": tok_real * self.world / dt,
                 "step_ms": dt * 1e3 / max(1, log_n)}
        if torch.cuda.is_available():
            extra["peak_hbm_gib"] = torch.cuda.max_memory_allocated() / 2 ** 30
        if self.args.wall_clock_breakdown:
            extra.update({f"{k}_ms": v / max(1, log_n) for k, v in self.timer.summary().items()})
        self.metrics.write(step=self.state.global_step, **rec, **extra)

    # ------------------------------------------------------------------ HF helpers
    def log_metrics(self, split, metrics):
        if self.rank != 0:
            return
        print(f"***** {split} metrics *****")
        for k in sorted(metrics):
            print(f"  {k:<28} = {metrics[k]}")

    def save_metrics(self, split, metrics, combined=True):
        if self.rank != 0:
            return
        os.makedirs(self.args.output_dir, exist_ok=True)
        with open(os.path.join(self.args.output_dir, f"{split}_results.json"), "w") as f:
            json.dump(metrics, f, indent=4)
        if combined:
            p = os.path.join(self.args.output_dir, "all_results.json")
            allm = json.load(open(p)) if os.path.exists(p) else {}
            allm.update(metrics)
            with open(p, "w") as f:
                json.dump(allm, f, indent=4)

    def save_state(self):
        if self.rank == 0:
            os.makedirs(self.args.output_dir, exist_ok=True)
            self.state.save_to_json(os.path.join(self.args.output_dir, "trainer_state.json"))

    def save_interrupted(self):
        """The reference's crash handler (``qwen3-8b-lora.py:190-204``): save the current
        adapter to ``<output_dir>_interrupted``."""
        d = self._interrupt_dir or self.args.output_dir.rstrip("/") + "_interrupted"
        self._save_weights(d)
        return d

    @torch.no_grad()
    def evaluate(self, eval_dataset=None):
        """Mean loss (+ ``compute_metrics(EvalPrediction(predictions, label_ids))`` when given,
        e.g. accuracy for ``HF_Basics/trainer_demo.py``); distributed: sums all-reduced."""
        ds = eval_dataset or self.eval_dataset
        self.model.eval()
        bs = self.args.per_device_eval_batch_size
        samp = _EpochSampler(len(ds), self.world, self.rank, 0, shuffle=False)
        idx = samp.indices(0)
        tot = torch.zeros(2, device=self.device, dtype=torch.float64)
        preds, labels = [], []
        for s in range(0, len(idx), bs):
            b = self._to_device(self.data_collator([ds[j] for j in idx[s:s + bs]]))
            if self.compute_metrics is not None and isinstance(b, dict):
                out = self.model(**b)
                loss = out.loss
                preds.append(out.logits.float().cpu())
                labels.append(b["labels"].cpu())
            else:
                loss = self.compute_loss(self.model, b)
            tot[0] += float(loss) * len(idx[s:s + bs])
            tot[1] += len(idx[s:s + bs])
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(tot)
        self.model.train()
        el = float(tot[0] / tot[1])
        res = {"eval_loss": el}
        if self.compute_metrics is not None and preds:
            p, l = torch.cat(preds), torch.cat(labels)
            if self.world > 1:
                import torch.distributed as dist
                gp = [None] * self.world
                dist.all_gather_object(gp, (p, l))
                p, l = torch.cat([x[0] for x in gp]), torch.cat([x[1] for x in gp])
            res.update({f"eval_{k}": v for k, v in self.compute_metrics(EvalPrediction(p, l)).items()})
        else:
            res["perplexity"] = math.exp(min(el, 50))
        return res

    def _eval_and_track(self):
        m = self.evaluate()
        m["epoch"] = round(self.state.epoch, 4)
        self.state.log_history.append(dict(m, step=self.state.global_step))
        self._last_eval = m
        if self.rank == 0:
            print(m, flush=True)

    def _track_best(self):
        a = self.args
        m = getattr(self, "_last_eval", None)
        if not m:
            return
        key = a.metric_for_best_model or "loss"
        key = key if key.startswith("eval_") else "eval_" + key
        if key not in m:
            return
        gib = a.greater_is_better if a.greater_is_better is not None else not key.endswith("loss")
        v = m[key]
        if self.state.best_metric is None or (v > self.state.best_metric if gib else v < self.state.best_metric):
            self.state.best_metric = v
            self.state.best_model_checkpoint = os.path.join(a.output_dir,
                                                            f"{PREFIX_CHECKPOINT_DIR}-{self.state.global_step}")

    def _load_weights_only(self, ck):
        m = _unwrap(self.model)
        if os.path.exists(os.path.join(ck, "adapter_model.safetensors")) and hasattr(m, "load_adapter"):
            m.load_adapter(ck)
        elif os.path.exists(os.path.join(ck, "model.safetensors")):
            from safetensors.torch import load_file
            sd = load_file(os.path.join(ck, "model.safetensors"))
            with torch.no_grad():
                own = m.state_dict()
                for k, v in sd.items():
                    if k in own:
                        own[k].copy_(v.to(own[k].device, own[k].dtype))


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
