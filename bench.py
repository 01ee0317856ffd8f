#!/usr/bin/env python3
"""Headline benchmark: Qwen3-8B QLoRA fine-tune throughput (tokens/s, whole node).

Config = the reference's ``Fine-Tuning/qwen3-8b-qlora-dist.py`` (BASELINE.json / BASELINE.md):
NF4 + double-quant base (compute bf16), LoRA r=8 / alpha=16 / dropout=0.1 on q_proj+v_proj,
per-device batch 2 × 512 tokens, gradient accumulation 2, paged-AdamW-8bit (lr 5e-5, linear
schedule), max_grad_norm 1.0, DDP over RCCL for N>1.  Synthetic random token ids and
random-init weights of the Qwen3-8B architecture (no checkpoint / dataset download).

Every timed step is a full optimizer step: GA forward+backward micro-steps, the DDP gradient
all-reduce, global-norm clipping and the 8-bit AdamW update.

    python bench.py --gpus 1 --steps 10 --warmup 3
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

Rank 0 prints ONE JSON line (value = aggregate tokens/s over all ranks, max time over ranks).
"""
import argparse
import contextlib
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config  # noqa: E402
from llm_in_practise_amd.optim.adamw import LRScheduler, build_optimizer  # noqa: E402
from llm_in_practise_amd.parallel import dist as D  # noqa: E402
from llm_in_practise_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4  # noqa: E402
from llm_in_practise_amd.utils.gc_control import ManualGC  # noqa: E402
from llm_in_practise_amd.utils.watchdog import Watchdog  # noqa: E402

BASELINE_TOKENS_PER_S = None   # the reference publishes no fine-tune throughput
MODEL_NAMES = {"qwen3-8b": "Qwen3-8B", "qwen3-14b": "Qwen3-14B", "qwen3-4b": "Qwen3-4B",
               "deepseek-r1-0528-qwen3-8b": "DeepSeek-R1-0528-Qwen3-8B", "qwen3-tiny": "qwen3-tiny",
               "qwen3-small": "qwen3-small"}


def log(*a):
    if D.is_main():
        print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(n: int) -> int:
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def _fault_injector(record: str, rank: int):
    """``LIPA_BENCH_FAULT=<record>=<rank>:<step>:<kind>[;...]`` (kinds: utils/faults.py) — a fault injected into one
    sub-record of the bench (faithful / selective / zero3) to test that the headline record survives it."""
    from llm_in_practise_amd.utils.faults import FaultInjector
    spec = ",".join(item.split("=", 1)[1] for item in os.environ.get("LIPA_BENCH_FAULT", "").split(";")
                    if item.startswith(record + "="))
    return FaultInjector(spec, rank=rank)


def build(args, device):
    cfg = qwen3_config(args.model)
    t0 = time.time()
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = Qwen3ForCausalLM.from_config(cfg, dtype=dtype, device=device, seed=1234)
    if args.mode == "qlora":
        quantize_model_nf4(model, double_quant=True, compute_dtype=dtype)
    lcfg = LoraConfig(r=args.lora_r, lora_alpha=args.lora_alpha, lora_dropout=args.lora_dropout,
                      target_modules=args.targets.split(","))
    pm = get_peft_model(model, lcfg)
    model.fuse_projections()
    if args.grad_ckpt:
        model.gradient_checkpointing_enable({"use_reentrant": bool(args.ckpt_reentrant), "policy": args.ckpt_policy})
    pm.train()
    if device.type == "cuda":
        torch.cuda.synchronize()
    log(f"[bench] built {args.model} ({args.mode}) in {time.time() - t0:.1f}s; "
        f"trainable={sum(p.numel() for p in pm.parameters() if p.requires_grad):,}")
    return cfg, pm


def zero3_subrecord(args, device, rank: int, world: int, sync, beat=lambda: None) -> dict:
    """BASELINE config #4 at world > 1: ``Fine-Tuning/qwen3-14b-qlora-dist-deepspeed.py:164`` + ``ds_zero3_config.json``
    — the QLoRA model (--zero3-model, Qwen3-14B by default) on the ZeRO-3 engine, the client paged 8-bit AdamW on
    each rank's partition, the same micro-batch / GA / sequence length as the headline, GA micro-batches fused
    into one pass (identical gradient).  Timed like the headline (barrier + synchronize on both sides, max over
    ranks) with the per-step collective record (all-gathers, reduce-scatters)."""
    import gc
    from llm_in_practise_amd.parallel.zero import ZeroEngine
    gc.collect()
    if device.type == "cuda":
        torch.cuda.empty_cache()
    sub = argparse.Namespace(**vars(args))
    sub.model = args.zero3_model or ("qwen3-14b" if device.type == "cuda" else args.model)
    cfg, model = build(sub, device)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs", "ds_zero3_config.json")
    with open(path) as f:
        ds = json.load(f)
    ds["gradient_accumulation_steps"] = 1
    ds["train_micro_batch_size_per_gpu"] = args.micro_batch * args.grad_accum
    ds["train_batch_size"] = args.micro_batch * args.grad_accum * world
    warm = 1
    engine = ZeroEngine(model, ds, lr=args.lr, weight_decay=0.0, hidden_size=cfg.hidden_size,
                        total_steps=warm + args.zero3_steps, optim=args.optim)
    gen = torch.Generator(device=device).manual_seed(2000 + rank)
    data = torch.randint(0, cfg.vocab_size, (args.micro_batch * args.grad_accum, args.seq_len), device=device,
                         generator=gen)

    def step():
        out = engine.module(data, labels=data, num_micro_batches=args.grad_accum)
        engine.backward(out.loss)
        loss = out.loss.detach()
        del out
        engine.step()
        return loss

    inj = _fault_injector("zero3", rank)
    for _ in range(warm):
        step()
        beat()
    sync()
    if device.type == "cuda":
        torch.cuda.reset_peak_memory_stats(device)
    D.COMM.reset()
    D.COMM.enabled = True
    t0 = time.perf_counter()
    for i in range(args.zero3_steps):
        inj.check(i)
        loss = step()
        D.COMM.step()
        beat()
    sync()
    el = D.all_reduce_max(time.perf_counter() - t0)
    D.COMM.enabled = False
    ms = 1000 * el / args.zero3_steps
    tps = args.micro_batch * args.seq_len * args.grad_accum * world * args.zero3_steps / el
    mem = torch.cuda.max_memory_allocated(device) / 2 ** 30 if device.type == "cuda" else 0.0
    log(f"[bench] zero3 {sub.model}: loss={loss.item():.4f} {ms:.1f} ms/step {tps:,.0f} tok/s peak HBM {mem:.1f} GiB")
    return {"model": MODEL_NAMES.get(sub.model, sub.model), "value": round(tps, 1), "unit": "tokens/s",
            "ms_per_step": round(ms, 2), "steps": args.zero3_steps, "warmup": warm, "n_gpus": world,
            "parallelism": f"zero3-dp{world}", "ds_config": "configs/ds_zero3_config.json",
            "optimizer": f"zero3-{engine.optim_name}", "global_batch": args.micro_batch * args.grad_accum * world,
            "ga_execution": "fused-pass", "peak_hbm_gib": round(mem, 1),
            "dist_backend": torch.distributed.get_backend(), "comm": D.COMM.summary()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="qwen3-8b")
    ap.add_argument("--mode", default="qlora", choices=["qlora", "lora"])
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--grad-accum", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--lora-r", type=int, default=8)
    ap.add_argument("--lora-alpha", type=int, default=16)
    ap.add_argument("--lora-dropout", type=float, default=0.1)
    ap.add_argument("--targets", default="q_proj,v_proj")
    ap.add_argument("--optim", default="paged_adamw_8bit")
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--grad-ckpt", action="store_true",
                    help="recompute each decoder layer in backward (the reference's 24 GB-GPU setting; "
                         "off by default: 288 GB HBM holds every activation)")
    ap.add_argument("--strategy", default="ddp", choices=["ddp", "zero3"],
                    help="ddp: flat-buffer DDP over RCCL (qwen3-8b-qlora-dist.py); zero3: the ZeRO-3 engine with "
                         "ds_zero3_config.json semantics (qwen3-14b-qlora-dist-deepspeed.py, BASELINE config #4)")
    ap.add_argument("--ds-config", dest="ds_config", default=None)
    ap.add_argument("--ga-fusion", type=int, default=1,
                    help="1: execute the grad-accum micro-batches in one pass (per-micro-batch loss "
                         "normalisation, identical gradient); 0: sequential micro-steps")
    ap.add_argument("--faithful-steps", type=int, default=5,
                    help="after the headline timing, time this many steps of the reference-faithful config "
                         "(gradient checkpointing on, sequential GA micro-steps) in the same process and report "
                         "them as the JSON's 'faithful' sub-record (0: skip; ddp strategy only)")
    ap.add_argument("--faithful-warmup", type=int, default=2)
    ap.add_argument("--ckpt-reentrant", type=int, default=0,
                    help="checkpoint form of the faithful sub-record (the reference passes use_reentrant=False)")
    ap.add_argument("--ckpt-policy", default="full", choices=["selective", "full"],
                    help="recompute policy of --grad-ckpt (the faithful sub-record is always full): full = the whole layer "
                         "recomputed in backward (HF gradient_checkpointing, the reference); selective = GEMM outputs "
                         "recorded in the first forward, norms / RoPE / attention recomputed")
    ap.add_argument("--nf4-gemm", default=None, choices=["auto", "w4", "expand"],
                    help="NF4 base GEMM form (ops/gemm.py _nf4_w4): auto = one bf16 expansion per step where the copy "
                         "is reused (forward + dX), the in-kernel NF4 dequant-GEMM elsewhere; w4 = the NF4 dequant-GEMM "
                         "everywhere (no bf16 copy of the base: the memory-lean QLoRA step); expand = always expand "
                         "(default: LIPA_NF4_GEMM, else auto)")
    ap.add_argument("--zero3-steps", type=int, default=3,
                    help="world > 1 (ddp strategy): after the headline, also time this many steps of BASELINE config #4 "
                         "(--zero3-model QLoRA on the ZeRO-3 engine with configs/ds_zero3_config.json, same GA / optimizer) "
                         "as the 'zero3' sub-record, with its per-step collective record (0: skip)")
    ap.add_argument("--zero3-model", default=None,
                    help="model of the zero3 sub-record (default: qwen3-14b on GPUs, the headline model on CPU)")
    ap.add_argument("--selective-steps", type=int, default=3,
                    help="after the faithful sub-record, time this many steps with the selective recompute policy "
                         "(GEMM outputs of the first forward kept, not recomputed) as the 'selective_ckpt' sub-record")
    ap.add_argument("--selective-reentrant", type=int, default=1,
                    help="the selective_ckpt sub-record's checkpoint form (1: reentrant, this framework's choice; the "
                         "faithful record follows --ckpt-reentrant, the reference's use_reentrant=False)")
    ap.add_argument("--host-steps", type=int, default=2,
                    help="after the timed steps, issue this many steps onto an idle device and record the host "
                         "launch time of one step (host_launch_ms; LIPA_HOST_PROFILE=<file> adds a cProfile of them)")
    ap.add_argument("--stall-timeout-s", type=float, default=900.0,
                    help="watchdog (utils/watchdog.py): no progress (model built, one step finished) for this long "
                         "during the headline -> diagnostic with every thread's stack, exit 3 (a collective stall must "
                         "not wait out the process group's 30-minute timeout)")
    ap.add_argument("--subrecord-budget-s", type=float, default=None,
                    help="time budget of each sub-record (host / faithful / selective / zero3); past it the headline "
                         "line is printed with '<record>': {'error': ...} and the process exits 0 "
                         "(default: 240 s, 420 s for the zero3 sub-record, which builds its own model)")
    args = ap.parse_args()
    from llm_in_practise_amd.ops import gemm as _lin
    if args.nf4_gemm is not None:        # else the LIPA_NF4_GEMM environment choice stands
        _lin._NF4_MODE = args.nf4_gemm
    args.nf4_gemm = _lin._NF4_MODE

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without a launcher: start N ranks under torch.distributed.run
        # as a CHILD process (nothing here has touched the GPU yet; never exec) and exit with its code
        sys.exit(_self_launch(args.gpus))
    rank, local_rank, world = D.init_distributed()
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    wd = Watchdog(rank)
    wd.arm(args.stall_timeout_s, "headline: build + warmup", exit_code=3)
    device = torch.device("cuda", D.local_device_index(local_rank)) if torch.cuda.is_available() else torch.device("cpu")
    cfg, model = build(args, device)
    wd.beat()
    total_steps = args.warmup + args.steps
    engine = None
    if args.strategy == "zero3":
        from llm_in_practise_amd.parallel.zero import ZeroEngine
        path = args.ds_config or os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs",
                                              "ds_zero3_config.json")
        with open(path) as f:
            ds = json.load(f)
        if args.ga_fusion:   # the GA micro-batches run as ONE pass: the engine sees one micro-step
            ds["gradient_accumulation_steps"] = 1
            ds["train_micro_batch_size_per_gpu"] = args.micro_batch * args.grad_accum
            ds["train_batch_size"] = args.micro_batch * args.grad_accum * world
        engine = ZeroEngine(model, ds, lr=args.lr, weight_decay=0.0, hidden_size=cfg.hidden_size,
                            total_steps=total_steps, optim=args.optim)
        opt = sched = ddp = None
    else:
        opt = build_optimizer(args.optim, [p for p in model.parameters() if p.requires_grad], args.lr,
                              weight_decay=0.0, max_grad_norm=1.0)
        sched = LRScheduler(opt, "linear", args.lr, total_steps)
        ddp = DistributedDataParallel(model, flat=opt.flat)

    gen = torch.Generator(device=device).manual_seed(1000 + rank)
    n_batches = 8
    data = torch.randint(0, cfg.vocab_size, (n_batches, args.micro_batch, args.seq_len), device=device,
                         generator=gen)
    it = [0]
    spent = [None]

    def step(fused=None):
        fused = args.ga_fusion if fused is None else fused
        if engine is not None:      # ZeRO-3: reduce-scatter / optimizer partition / clip inside step()
            ids = torch.cat([data[(it[0] + g) % n_batches] for g in range(args.grad_accum)])
            it[0] += args.grad_accum
            out = engine.module(ids, labels=ids, num_micro_batches=args.grad_accum if args.ga_fusion else 1)
            engine.backward(out.loss)
            loss = out.loss.detach()
            del out                 # tear the autograd graph down while the GPU still runs the backward
            engine.step()
            return loss
        if fused:
            # the GA micro-batches are independent given the (frozen-during-the-step) weights:
            # run them as one pass with per-micro-batch loss normalisation (same gradient)
            ids = torch.cat([data[(it[0] + g) % n_batches] for g in range(args.grad_accum)])
            it[0] += args.grad_accum
            out = model(ids, labels=ids, num_micro_batches=args.grad_accum)
            # the previous step's spent autograd graph (~2k nodes) is torn down here, while this
            # forward is queued on the GPU; released at `loss = step()` the teardown left the GPU
            # idle ~0.9 ms per step (profiles/bench_qwen3_8b_qlora_step_timeline_v12.txt)
            spent[0] = None
            out.loss.backward()
            loss = out.loss.detach()
            spent[0] = out
        else:
            for micro in range(args.grad_accum):
                ids = data[it[0] % n_batches]
                it[0] += 1
                ctx = ddp.no_sync() if micro < args.grad_accum - 1 else contextlib.nullcontext()
                with ctx:
                    out = model(ids, labels=ids)
                    spent[0] = None         # the previous micro-step's graph, torn down under this forward
                    (out.loss / args.grad_accum).backward()
                loss = out.loss.detach()
                spent[0] = out
        ddp.allreduce_grads()
        opt.clip_grad_norm_(1.0)
        opt.step()
        sched.step()
        opt.zero_grad()
        return loss

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()
        D.barrier()

    for i in range(args.warmup):
        loss = step()
        wd.beat()
        if i == 0:
            sync()
            log(f"[bench] first step done, loss={loss.item():.4f}")
    sync()
    if device.type == "cuda":     # peak HBM of the training steps (not of building / quantising the model)
        torch.cuda.reset_peak_memory_stats(device)
    gcm = ManualGC().__enter__()    # automatic Python GC off, a full pass every LIPA_GC_INTERVAL steps (utils/gc_control.py)
    D.COMM.reset()
    D.COMM.enabled = world > 1      # collectives of the timed steps: bytes, run time, exposed time (parallel/dist.py)
    _lin.GEMM_STATS.clear()         # GEMM launches by form over the timed steps (kernel provenance)
    t0 = time.perf_counter()
    dbg = os.environ.get("LIPA_BENCH_DEBUG_LOSS") == "1"     # per-step loss / grad norm (syncs: debug only)
    wd.arm(args.stall_timeout_s, "headline: timed steps", exit_code=3)
    for _ in range(args.steps):
        loss = step()
        gcm.step()
        D.COMM.step()
        wd.beat()
        if dbg:
            gn = getattr(engine, "last_grad_norm", None) if engine is not None else None
            print(f"[rank {rank}] step loss={loss.item():.6f} grad_norm={None if gn is None else float(gn):}",
                  file=sys.stderr, flush=True)
    sync()
    elapsed = D.all_reduce_max(time.perf_counter() - t0)
    wd.disarm()
    D.COMM.enabled = False
    comm = D.COMM.summary() if world > 1 else None
    gemm_forms = {k: round(v / max(1, args.steps), 2) for k, v in sorted(_lin.GEMM_STATS.items())}
    ms = 1000 * elapsed / max(1, args.steps)
    tokens = args.micro_batch * args.seq_len * args.grad_accum * world * args.steps
    tps = tokens / elapsed
    nonpad_frac = 1.0                # random ids: no pad token, every label position counts
    lin = cfg.num_params() - cfg.vocab_size * cfg.hidden_size * (1 if cfg.tie_word_embeddings else 2)
    head = cfg.vocab_size * cfg.hidden_size
    # fwd 2·(linear+head) + bwd dX 2·(linear+head); no weight grads for the frozen base
    fl_per_tok = 4 * (lin + head) * (1.5 if args.grad_ckpt else 1.0)
    mem = torch.cuda.max_memory_allocated(device) / 2 ** 30 if device.type == "cuda" else 0.0
    log(f"[bench] loss={loss.item():.4f} {ms:.1f} ms/step  {tps:,.0f} tok/s  "
        f"~{tps * fl_per_tok / world / 1e12:.0f} TFLOP/s/GPU (matmul)  peak HBM {mem:.1f} GiB")

    # ---- the headline record, complete before any sub-record runs (every rank holds it; rank 0 prints it)
    rec = {
        "metric": f"tokens/sec (whole node) {MODEL_NAMES.get(args.model, args.model)} "
                  f"{'QLoRA' if args.mode == 'qlora' else 'LoRA'} fine-tune at 1/2/4/8 MI355X",
        "value": round(tps, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 2),
        "host_launch_ms": None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(tps / BASELINE_TOKENS_PER_S, 3) if BASELINE_TOKENS_PER_S else None),
        "dtype": "bf16" if device.type == "cuda" else "fp32",
        "data": "synthetic",
        "config": {
            "model": MODEL_NAMES.get(args.model, args.model),
            "global_batch": args.micro_batch * args.grad_accum * world,
            "seq_len": args.seq_len,
            "parallelism": f"dp{world}" if engine is None else f"zero3-dp{world}",
            "micro_batch": args.micro_batch,
            "grad_accum": args.grad_accum,
            "quant": "nf4+double_quant" if args.mode == "qlora" else "none",
            "nf4_gemm": args.nf4_gemm,
            # kernel provenance of the timed steps (ops/gemm.py GEMM_STATS): GEMM launches per step by form —
            # gemm4w = the hand-written HIP GEMM on a bf16 operand, gemm4w-nf4 = the same kernel reading NF4 codes,
            # library = torch.matmul (shapes gemm4w does not take); nf4-expansion = bf16 copies of NF4 bases
            "gemm_backend": "gemm4w" if device.type == "cuda" else "torch-cpu",
            "gemm_launches_per_step": {k: v for k, v in gemm_forms.items() if k != "nf4-expansion"},
            "nf4_expansions_per_step": gemm_forms.get("nf4-expansion", 0),
            "lora": f"r{args.lora_r}/a{args.lora_alpha}/drop{args.lora_dropout}/{args.targets}",
            "optimizer": args.optim if engine is None else f"zero3-{engine.optim_name}",
            "gradient_checkpointing": bool(args.grad_ckpt),
            "ga_execution": "fused-pass" if args.ga_fusion else "sequential",
            "weights": "random-init",
            "peak_hbm_gib": round(mem, 1),
            "dist_backend": (torch.distributed.get_backend() if D.is_dist() else "none"),
            "dist_world_size": D.world_size(),
            # padded = micro x 512 x GA x world / step; non-pad counts only label != -100 positions
            # (synthetic ids carry no padding, so the two agree here)
            "tokens_per_s_padded": round(tps, 1),
            "tokens_per_s_nonpad": round(tps * nonpad_frac, 1),
        },
        "comm": dict(comm, **D.comm_environment()) if comm is not None else {"skipped": "single rank: no collectives"},
    }
    if world == 1:
        rec["zero3"] = {"skipped": "single rank (the ZeRO-3 sub-record runs when world > 1)"}

    emitted = [False]
    emit_lock = threading.Lock()

    def emit():
        with emit_lock:
            if not emitted[0]:
                emitted[0] = True
                if D.is_main():
                    print(json.dumps(rec), flush=True)

    # ---- sub-records, each fault-isolated: an exception becomes '<key>': {'error': ...}; a stall (no progress for
    # the budget) prints the headline line with that error from the watchdog and exits 0.  After a failure at
    # world > 1 this rank issues no further collective (its peers may still be inside one): the remaining
    # sub-records are skipped and the process ends without the final barrier.
    poisoned = [False]
    budget_default = args.subrecord_budget_s or 240.0

    def sub(key, fn, budget_s=None):
        budget_s = budget_s or budget_default
        if poisoned[0]:
            rec[key] = {"skipped": "an earlier sub-record failed on this rank"}
            return None

        def expire():
            rec[key] = {"error": f"watchdog: no progress for {budget_s:.0f} s (collective stall, dead peer or hang)"}
            emit()
        wd.arm(budget_s, f"sub-record {key}", on_expire=expire, exit_code=0)
        try:
            out = fn(wd.beat)
        except Exception as e:   # noqa: BLE001 - every failure of a sub-record is recorded, none ends the run
            import traceback
            traceback.print_exc()
            rec[key] = {"error": f"{type(e).__name__}: {e}"[:600]}
            poisoned[0] = world > 1
            if device.type == "cuda":
                torch.cuda.empty_cache()
            return None
        finally:
            wd.disarm()
        if out is not None:
            rec[key] = out
        return out

    # host launch cost of one headline step (untimed, after the timed steps): the step is issued onto an idle
    # device and timed until step() returns — how far the Python/launch side is from becoming the bottleneck
    def host_record(beat):
        prof = None
        if os.environ.get("LIPA_HOST_PROFILE"):
            import cProfile
            prof = cProfile.Profile()
        hs = []
        for _ in range(args.host_steps):
            sync()
            h0 = time.perf_counter()
            if prof is not None:
                prof.enable()
            step()
            if prof is not None:
                prof.disable()
            hs.append(time.perf_counter() - h0)
            gcm.step()
            beat()
        sync()
        host_ms = round(1000 * min(hs), 2)
        log(f"[bench] host launch time of one step: {host_ms:.1f} ms (device {ms:.1f} ms/step)")
        if prof is not None and D.is_main():
            import pstats
            with open(os.environ["LIPA_HOST_PROFILE"], "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(60)
        rec["host_launch_ms"] = host_ms
        return None

    def timed_ckpt(policy: str, n_steps: int, reentrant: bool, beat) -> dict:
        """BASELINE.md's config as the reference runs it (Fine-Tuning/qwen3-8b-qlora-dist.py:137-138, 162-163):
        gradient checkpointing on and the GA micro-steps one after another (no_sync on all but the last), same
        model / optimizer / data, timed the same way as the headline.  policy "full" = HF's whole-layer
        recompute (use_reentrant=False, as the reference passes); "selective" = this framework's cheaper recompute,
        in the reentrant form by default (no saved-tensor pack / unpack hooks: ~20 ms less host time per step,
        which the selective step — 73 ms of GPU work — would otherwise wait on)."""
        inj = _fault_injector("faithful" if policy == "full" else "selective", rank)
        model.gradient_checkpointing_enable({"use_reentrant": reentrant, "policy": policy})
        for _ in range(args.faithful_warmup):
            step(fused=0)
            beat()
        sync()
        if device.type == "cuda":
            torch.cuda.reset_peak_memory_stats(device)
        tf0 = time.perf_counter()
        for i in range(n_steps):
            inj.check(i)
            floss = step(fused=0)
            gcm.step()
            beat()
        sync()
        fel = D.all_reduce_max(time.perf_counter() - tf0)
        fms = 1000 * fel / n_steps
        ftps = args.micro_batch * args.seq_len * args.grad_accum * world * n_steps / fel
        fmem = torch.cuda.max_memory_allocated(device) / 2 ** 30 if device.type == "cuda" else 0.0
        fhost = None
        if args.host_steps > 0:     # host issue time of one such step onto an idle device (untimed, after)
            prof = None
            if os.environ.get("LIPA_HOST_PROFILE_CKPT") == policy:   # cProfile it, backward on this thread
                import cProfile
                prof = cProfile.Profile()
                torch.autograd.set_multithreading_enabled(False)
            hs = []
            for k in range(args.host_steps):     # min over host_steps issues, as the headline's host record
                sync()
                h0 = time.perf_counter()
                if prof is not None and k == 0:
                    prof.enable()
                step(fused=0)
                if prof is not None and k == 0:
                    prof.disable()
                hs.append(time.perf_counter() - h0)
                gcm.step()
                beat()
            sync()
            fhost = round(1000 * min(hs), 2)
            if prof is not None:
                torch.autograd.set_multithreading_enabled(True)
                if D.is_main():
                    import pstats
                    with open(os.environ.get("LIPA_HOST_PROFILE", "host_profile_ckpt.txt"), "w") as f:
                        pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(50)
                        pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(40)
        log(f"[bench] grad ckpt ({policy}) + sequential GA: loss={floss.item():.4f} {fms:.1f} ms/step  "
            f"{ftps:,.0f} tok/s  peak HBM {fmem:.1f} GiB  host {fhost} ms/step")
        return {"value": round(ftps, 1), "unit": "tokens/s", "ms_per_step": round(fms, 2), "host_launch_ms": fhost,
                "steps": n_steps, "warmup": args.faithful_warmup,
                "gradient_checkpointing": True, "ga_execution": "sequential",
                "gradient_checkpointing_kwargs": {"use_reentrant": reentrant},
                "checkpoint_policy": policy,
                "micro_batch": args.micro_batch, "grad_accum": args.grad_accum, "peak_hbm_gib": round(fmem, 1)}

    if args.host_steps > 0:
        sub("host_launch_ms", host_record)
    if engine is None and not (args.grad_ckpt and not args.ga_fusion):
        if args.faithful_steps > 0:
            sub("faithful", lambda beat: timed_ckpt("full", args.faithful_steps, bool(args.ckpt_reentrant), beat))
        if args.selective_steps > 0:
            sub("selective_ckpt",
                lambda beat: timed_ckpt("selective", args.selective_steps, bool(args.selective_reentrant), beat))

    if world > 1 and engine is None and args.zero3_steps > 0 and poisoned[0]:
        rec["zero3"] = {"skipped": "an earlier sub-record failed on this rank"}
    elif world > 1 and engine is None and args.zero3_steps > 0:
        del step, timed_ckpt, host_record
        model = opt = sched = ddp = data = None
        spent[0] = None
        sub("zero3", lambda beat: zero3_subrecord(args, device, rank, world, sync, beat),
            args.subrecord_budget_s or 420.0)
    gcm.__exit__(None, None, None)
    emit()
    if poisoned[0]:
        # a peer may still be inside a collective of the failed sub-record: no barrier / destroy from here
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    wd.arm(120.0, "shutdown", exit_code=0)
    D.destroy()
    wd.disarm()


if __name__ == "__main__":
    main()
