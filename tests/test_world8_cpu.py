"""8-rank readiness on CPU (gloo): the driver's scaling run is the first time the code meets W=8 on
GPUs, so every world-size-dependent path is rehearsed here at W=4 and W=8 first.

* DDP bucket overlap: 8 ranks, buckets issued in the same (index) order on every rank, trained
  weights equal the single-process oracle on the concatenated batch
  (``ddp_basics/ddp_gpt_wikitext2.py:274`` semantics);
* ZeRO-1/2/3 with shards that do not divide evenly (40x40 blocks, biases) at W=8;
* ZeRO-3 checkpoint re-partitioning 8 -> 2 -> 8 (``zero_pp_rank_*`` shards, repartition-on-load);
* the custom peer all-reduce's host model (one-shot / two-shot / RCCL fallback) at W=8;
* ``bench.py --gpus 8`` self-launching 8 ranks (``Fine-Tuning/README.md:128-134`` launch contract).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

from llm_in_practise_amd.optim.adamw import AdamW
from llm_in_practise_amd.parallel.ddp import DistributedDataParallel
from llm_in_practise_amd.parallel.zero import ZeroEngine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W8 = 8


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1")
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)


class Net(nn.Module):
    def __init__(self, d=40, n=5):
        super().__init__()
        self.inp = nn.Linear(8, d)
        self.blocks = nn.ModuleList([nn.Sequential(nn.Linear(d, d), nn.Tanh()) for _ in range(n)])
        self.out = nn.Linear(d, 1)

    def forward(self, x):
        h = self.inp(x)
        for b in self.blocks:
            h = h + b(h)
        return self.out(h)


def _data(step, rank, n=2):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(n, 8, generator=g), torch.randn(n, 1, generator=g)


def _batch(step, world):
    xs, ys = zip(*[_data(step, r) for r in range(world)])
    return torch.cat(xs), torch.cat(ys)


# ----------------------------------------------------------------------------- DDP at W=8
def _ddp_worker(rank, world, port, out):
    _init(rank, world, port)
    torch.manual_seed(0)
    net = Net()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    ddp = DistributedDataParallel(net, flat=opt.flat, bucket_mb=0.004)
    logs = []
    for s in range(3):
        x, y = _data(s, rank)
        ((ddp(x) - y) ** 2).mean().backward()
        ddp.allreduce_grads()
        logs.append([b for b, _ in ddp.launch_log])
        ddp.reset_log()
        opt.step()
        opt.zero_grad()
    torch.save({"sd": net.state_dict(), "logs": logs, "nb": len(ddp._buckets)}, out.format(rank))
    torch.distributed.destroy_process_group()


def test_ddp_bucket_overlap_world8(tmp_path):
    out = str(tmp_path / "ddp{}.pt")
    mp.spawn(_ddp_worker, args=(W8, _port(), out), nprocs=W8, join=True)
    torch.manual_seed(0)
    net = Net()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    for s in range(3):
        x, y = _batch(s, W8)
        ((net(x) - y) ** 2).mean().backward()
        opt.step()
        opt.zero_grad()
    want = net.state_dict()
    for r in range(W8):
        got = torch.load(out.format(r), weights_only=True)
        assert got["nb"] >= 4
        for log in got["logs"]:
            assert log == list(range(got["nb"]))       # every rank, every step: index order
        for k, v in want.items():
            assert torch.allclose(got["sd"][k], v, atol=1e-5), (r, k)


# ----------------------------------------------------------------------------- ZeRO at W=8
def _cfg(stage):
    return {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1, "gradient_clipping": 0.05,
            "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}},
            "zero_optimization": {"stage": stage}}


def _zero_worker(rank, world, port, stage, out, steps=3, start=0, load=None, save=None):
    _init(rank, world, port)
    torch.manual_seed(0)
    eng = ZeroEngine(Net(), _cfg(stage))
    if load:
        eng.load_checkpoint(load)
    for s in range(start, start + steps):
        x, y = _data(s, rank) if world == W8 else [t.view(world, -1, t.shape[-1])[rank] for t in _batch(s, W8)]
        eng.backward(((eng(x) - y) ** 2).mean())
        eng.step()
    if save:
        eng.save_checkpoint(save)
    sd = eng.consolidated_state_dict()
    if rank == 0:
        torch.save(sd, out)
    torch.distributed.destroy_process_group()


def _zero_oracle(steps):
    torch.manual_seed(0)
    eng = ZeroEngine(Net(), _cfg(0))
    for s in range(steps):
        x, y = _batch(s, W8)
        eng.backward(((eng(x) - y) ** 2).mean())
        eng.step()
    return eng.module.state_dict()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_zero_uneven_shards_world8(tmp_path, stage):
    """Net's 40x40 blocks (1640 params per unit) and 1-row head do not split evenly over 8 ranks."""
    out = str(tmp_path / "z.pt")
    mp.spawn(_zero_worker, args=(W8, _port(), stage, out), nprocs=W8, join=True)
    got, want = torch.load(out, weights_only=True), _zero_oracle(3)
    for k in want:
        assert torch.allclose(got[k], want[k], atol=2e-5), (stage, k, (got[k] - want[k]).abs().max())


def test_zero3_checkpoint_repartition_8_2_8(tmp_path):
    """Train 2 steps at W=8, resume 1 step at W=2, resume 1 step at W=8: equals 4 uninterrupted steps."""
    ck1, ck2 = str(tmp_path / "ck8"), str(tmp_path / "ck2")
    mp.spawn(_zero_worker, args=(W8, _port(), 3, str(tmp_path / "a.pt"), 2, 0, None, ck1), nprocs=W8, join=True)
    mp.spawn(_zero_worker, args=(2, _port(), 3, str(tmp_path / "b.pt"), 1, 2, ck1, ck2), nprocs=2, join=True)
    mp.spawn(_zero_worker, args=(W8, _port(), 3, str(tmp_path / "c.pt"), 1, 3, ck2, None), nprocs=W8, join=True)
    got, want = torch.load(str(tmp_path / "c.pt"), weights_only=True), _zero_oracle(4)
    for k in want:
        assert torch.allclose(got[k], want[k], atol=2e-5), (k, (got[k] - want[k]).abs().max())


# ----------------------------------------------------------------------------- custom all-reduce W=8
def _car_worker(rank, world, port, q):
    _init(rank, world, port)
    from llm_in_practise_amd.parallel.custom_allreduce import CustomAllReduce
    car = CustomAllReduce(backend="host", max_bytes=64 << 10, one_shot_bytes=4 << 10)
    try:
        ok = []
        for step, n in enumerate([64, 1000, 4096, 12000, 30000]):     # 256 B .. 120 KB (> cap: RCCL/gloo)
            g = torch.Generator().manual_seed(step * 100 + rank)
            t = torch.randn(n, generator=g)
            ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(step * 100 + r)) for r in range(world))
            car.all_reduce_(t)
            ok.append(bool(torch.allclose(t, ref, atol=1e-4, rtol=1e-5)))
        q.put((rank, ok, dict(car.calls)))
    finally:
        car.close()
        torch.distributed.destroy_process_group()


def test_custom_allreduce_host_model_world8():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_car_worker, args=(r, W8, port, q)) for r in range(W8)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(W8)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok, calls in res:
        assert all(ok), (rank, ok)
        assert calls == {"oneshot": 2, "twoshot": 2, "fallback": 1}, calls


# ----------------------------------------------------------------------------- DDP all-reduce policy at W=8
def test_allreduce_path_policy():
    from llm_in_practise_amd.parallel.ddp import ONE_SHOT_BYTES, allreduce_path
    assert allreduce_path(4096, 1, True) == "none"
    assert allreduce_path(4096, 8, True) == "peer-oneshot"
    assert allreduce_path(ONE_SHOT_BYTES, 8, True) == "peer-oneshot"
    assert allreduce_path(ONE_SHOT_BYTES + 16, 8, True) == "rccl"
    assert allreduce_path(4096, 8, False) == "rccl"           # multi-node: RCCL
    assert allreduce_path(4100, 8, True) == "rccl"            # not 16-B granular
    assert allreduce_path(15 << 20, 8, True) == "rccl"        # the QLoRA headline's adapter-gradient sizes


def _ddp_policy_worker(rank, world, port, out):
    _init(rank, world, port)
    torch.manual_seed(0)
    big = Net(d=260, n=2)              # ~137k params: 2 buckets of ~68k floats (270 KB > 256 KiB) ...
    small = Net(d=16, n=2)             # ... and one small model whose buckets are latency-bound
    res = {}
    for name, net, mb in (("big", big, 0.26), ("small", small, 0.004)):
        opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
        ddp = DistributedDataParallel(net, flat=opt.flat, bucket_mb=mb, custom_allreduce="auto-host")
        for s in range(2):
            x, y = _data(s, rank)
            ((ddp(x) - y) ** 2).mean().backward()
            ddp.allreduce_grads()
            opt.step()
            opt.zero_grad()
        res[name] = (None if ddp.car is None else dict(ddp.car.calls), {k: v.clone() for k, v in net.state_dict().items()})
        ddp.close()
    torch.save(res, out.format(rank))
    torch.distributed.destroy_process_group()


def test_ddp_allreduce_policy_world8(tmp_path):
    """8 ranks: DDP's "auto" all-reduce sends only the ≤ 256 KiB buckets through the peer-memory one-shot
    (here its /dev/shm host model) and builds no peer path at all when every bucket is larger (the
    QLoRA headline); both train to the single-process oracle."""
    out = str(tmp_path / "pol{}.pt")
    mp.spawn(_ddp_policy_worker, args=(W8, _port(), out), nprocs=W8, join=True)
    for name, net in (("big", Net(d=260, n=2)), ("small", Net(d=16, n=2))):
        pass
    got = [torch.load(out.format(r), weights_only=True) for r in range(W8)]
    assert all(g["big"][0] is None for g in got)                     # no bucket small enough: RCCL only
    for g in got:
        calls = g["small"][0]
        assert calls is not None and calls["oneshot"] > 0 and calls["twoshot"] == 0 and calls["fallback"] == 0
    for name, d in (("big", 260), ("small", 16)):
        torch.manual_seed(0)
        if name == "small":
            Net(d=260, n=2)                                            # same RNG consumption as the workers
        net = Net(d=d, n=2)
        opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
        for s in range(2):
            x, y = _batch(s, W8)
            ((net(x) - y) ** 2).mean().backward()
            opt.step()
            opt.zero_grad()
        for r in range(W8):
            for k, v in net.state_dict().items():
                assert torch.allclose(got[r][name][1][k], v, atol=1e-5), (name, r, k)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("lipa_car_")]


# ----------------------------------------------------------------------------- ZeRO-3 frozen NF4 partition
def _qlora_tiny():
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4
    cfg = qwen3_config("qwen3-tiny")
    m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0)
    quantize_model_nf4(m, compute_dtype=torch.float32)
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    torch.manual_seed(1)
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.05)
    m.fuse_projections()
    return pm, m, cfg


def _nf4_part_worker(rank, world, port, part, out):
    from llm_in_practise_amd.quant.nf4 import dequantize_nf4
    _init(rank, world, port)
    pm, m, cfg = _qlora_tiny()
    gu0 = dequantize_nf4(m.model.layers[0].mlp._gu.base, torch.float32).clone()
    down0 = m.model.layers[1].mlp.down_proj.weight.clone()        # Linear4bit: dequantised view
    ds = {"train_micro_batch_size_per_gpu": 1, "gradient_accumulation_steps": 1,
          "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.0}},
          "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0,
                                "stage3_partition_frozen_quant": part}}
    eng = ZeroEngine(pm, ds)
    res = {}
    for s in range(2):
        g = torch.Generator().manual_seed(100 * s + rank)
        ids = torch.randint(0, cfg.vocab_size, (1, 16), generator=g)
        loss = eng(ids, labels=ids).loss
        eng.backward(loss)
        eng.step()
        res[f"loss{s}"] = loss.detach()
    quant = [u.quant for u in eng.units if u.quant is not None]
    if part:
        assert len(quant) == cfg.num_hidden_layers
        for q in quant:       # released: this rank holds only its 1/W of the unit's quantised bytes
            assert q.full.untyped_storage().nbytes() == 0
            assert all(t.untyped_storage().nbytes() == 0 for t in q.tensors)
            assert q.shard.numel() * world == q.npad and q.shard.numel() % 512 == 0
        res["shard_bytes"] = torch.tensor(sum(q.shard.numel() for q in quant))
    else:
        assert not quant
    with eng.gathered_params():   # bit-identical bases after gather (fused view and Linear4bit buffers)
        assert torch.equal(dequantize_nf4(m.model.layers[0].mlp._gu.base, torch.float32), gu0)
        assert torch.equal(m.model.layers[1].mlp.down_proj.weight, down0)
    sd = eng.consolidated_state_dict()
    res.update({k: v for k, v in sd.items() if "lora_" in k or k.endswith("codes")})
    torch.save(res, out.format(rank))
    torch.distributed.destroy_process_group()


def test_zero3_partitions_frozen_nf4_world8(tmp_path):
    """SURVEY §7.5.3 option 1 (qwen3-14b-qlora-dist-deepspeed.py:164 under ds_zero3_config.json): the
    frozen NF4 bases are sharded by whole quant blocks over 8 ranks and all-gathered per layer unit;
    the training trajectory equals the replicated-base run exactly."""
    outs = {}
    for part in (False, True):
        out = str(tmp_path / f"p{int(part)}_{{}}.pt")
        mp.spawn(_nf4_part_worker, args=(W8, _port(), part, out), nprocs=W8, join=True)
        outs[part] = [torch.load(out.format(r), weights_only=True) for r in range(W8)]
    for r in range(W8):
        a, b = outs[False][r], outs[True][r]
        for k in a:
            assert torch.equal(a[k], b[k]), (r, k)
    assert any("lora_B" in k for k in outs[True][0])
    full = sum(v.numel() for k, v in outs[True][0].items() if k.endswith("codes"))
    assert outs[True][0]["shard_bytes"].item() < full / W8 * 1.2     # 1/8 of codes + scales + padding


# ----------------------------------------------------------------------------- bench.py --gpus 8
def test_bench_self_launches_eight_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
           "--model", "qwen3-tiny", "--seq-len", "32"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["dist_world_size"] == 8 and d["config"]["parallelism"] == "dp8"
    assert d["config"]["global_batch"] == 8 * d["config"]["micro_batch"] * d["config"]["grad_accum"]
