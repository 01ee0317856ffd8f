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
