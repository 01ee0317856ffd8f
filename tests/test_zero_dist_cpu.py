"""ZeRO-0/1/2/3 (+offload, fp16 scaler) equivalence on CPU with gloo, world_size 2.

Oracle: the same model trained in ONE process on the concatenation of both ranks' batches
(mean loss) — data parallelism with averaged gradients must reproduce it for every stage.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

from llm_in_practise_amd.parallel.zero import LossScaler, ZeroEngine, initialize
from llm_in_practise_amd.parallel.ds_config import load_ds_config


class Net(nn.Module):
    def __init__(self, d=16, n=3):
        super().__init__()
        self.inp = nn.Linear(8, d)
        self.blocks = nn.ModuleList([nn.Sequential(nn.Linear(d, d), nn.Tanh()) for _ in range(n)])
        self.out = nn.Linear(d, 1)

    def forward(self, x):
        h = self.inp(x)
        for b in self.blocks:
            h = h + b(h)
        return self.out(h)


def _data(step, rank, n=4):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(n, 8, generator=g), torch.randn(n, 1, generator=g)


def _cfg(stage, offload=False, clip=0.05, ga=1):
    z = {"stage": stage}
    if offload:
        z["offload_optimizer"] = {"device": "cpu"}
    return {"train_micro_batch_size_per_gpu": 4, "gradient_accumulation_steps": ga, "gradient_clipping": clip,
            "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}},
            "zero_optimization": z}


def _train(engine, world, rank, steps=3, ga=1):
    for s in range(steps):
        for mstep in range(ga):
            x, y = _data(s * ga + mstep, rank)
            loss = ((engine(x) - y) ** 2).mean()
            engine.backward(loss)
            engine.step()


def _worker(rank, world, port, stage, offload, ga, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = Net()
    eng = ZeroEngine(net, _cfg(stage, offload, ga=ga))
    _train(eng, world, rank, ga=ga)
    sd = eng.consolidated_state_dict()
    if rank == 0:
        torch.save(sd, out)
    torch.distributed.destroy_process_group()


def _oracle(steps=3, ga=1, n=3):
    torch.manual_seed(0)
    net = Net(n=n)
    eng = ZeroEngine(net, _cfg(0, ga=ga))
    for s in range(steps):
        for mstep in range(ga):
            xs, ys = zip(*[_data(s * ga + mstep, r) for r in range(2)])
            loss = ((eng(torch.cat(xs)) - torch.cat(ys)) ** 2).mean()
            eng.backward(loss)
            eng.step()
    return net.state_dict()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("stage,offload,ga", [(0, False, 1), (1, False, 1), (2, False, 2), (3, False, 1),
                                               (3, False, 2), (2, True, 1)])
def test_zero_stage_matches_single_process(tmp_path, stage, offload, ga):
    if offload:
        from llm_in_practise_amd.ops._native import cpu_native
        cpu_native()
    out = str(tmp_path / "sd.pt")
    mp.spawn(_worker, args=(2, _free_port(), stage, offload, ga, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want = _oracle(ga=ga)
    for k in want:
        assert torch.allclose(got[k], want[k], atol=2e-5), (stage, k, (got[k] - want[k]).abs().max())


def _ckpt_worker(rank, world, port, d, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    eng = ZeroEngine(Net(), _cfg(2))
    _train(eng, world, rank, steps=2)
    eng.save_checkpoint(d, client_state={"epoch": 1})
    torch.manual_seed(123)                       # different init: load must restore everything
    eng2 = ZeroEngine(Net(), _cfg(2))
    _, client = eng2.load_checkpoint(d)
    for e in (eng, eng2):
        x, y = _data(99, rank)
        e.backward(((e(x) - y) ** 2).mean())
        e.step()
    a, b = eng.consolidated_state_dict(), eng2.consolidated_state_dict()
    if rank == 0:
        torch.save({"ok": all(torch.equal(a[k], b[k]) for k in a), "client": client["epoch"],
                    "files": sorted(os.listdir(os.path.join(d, "global_step2")))}, out)
    torch.distributed.destroy_process_group()


def test_zero_checkpoint_roundtrip(tmp_path):
    out = str(tmp_path / "r.pt")
    mp.spawn(_ckpt_worker, args=(2, _free_port(), str(tmp_path / "ck"), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    assert r["ok"] and r["client"] == 1
    assert r["files"] == ["mp_rank_00_model_states.pt", "zero_pp_rank_0_mp_rank_00_optim_states.pt",
                          "zero_pp_rank_1_mp_rank_00_optim_states.pt"]
    assert open(tmp_path / "ck" / "latest").read() == "global_step2"


def test_stage3_single_process_frees_and_regathers():
    torch.manual_seed(0)
    net = Net(d=64)
    eng = ZeroEngine(net, {"zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 10},
                           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}})
    blocks = [u for u in eng.units if u.module is not net]
    assert blocks and all(not u.gathered for u in blocks)
    x, y = _data(0, 0)
    eng.backward(((eng(x) - y) ** 2).mean())
    assert all(not u.gathered for u in blocks)
    eng.step()
    assert float(eng.grad_shard.abs().sum()) == 0.0


def test_loss_scaler_dynamics():
    cfg = load_ds_config({"fp16": {"enabled": True, "loss_scale": 0, "initial_scale_power": 4,
                                   "loss_scale_window": 2, "hysteresis": 1, "min_loss_scale": 1}})
    s = LossScaler(cfg)
    assert s.scale == 16
    s.update(True)
    assert s.scale == 8
    s.update(False)
    s.update(False)
    assert s.scale == 16


def test_fp16_overflow_skips_step():
    torch.manual_seed(0)
    net = Net()
    eng = ZeroEngine(net, {"fp16": {"enabled": True, "initial_scale_power": 4, "hysteresis": 1},
                           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}, "zero_optimization": {"stage": 1}})
    before = {k: v.clone() for k, v in net.state_dict().items()}
    x, y = _data(0, 0)
    loss = ((eng(x.half()) - y.half()) ** 2).mean() * float("inf")
    eng.backward(loss)
    eng.step()
    assert eng.skipped_steps == 1 and eng.scaler.scale == 8
    assert all(torch.equal(before[k], v) for k, v in net.state_dict().items())


def test_ds_config_auto_resolution_and_validation():
    c = load_ds_config({"train_batch_size": "auto", "train_micro_batch_size_per_gpu": "auto",
                        "gradient_accumulation_steps": "auto",
                        "zero_optimization": {"stage": 3, "reduce_bucket_size": "auto",
                                              "stage3_prefetch_bucket_size": "auto",
                                              "stage3_param_persistence_threshold": "auto"}},
                       world_size=4, micro_batch=2, grad_accum=8, hidden_size=4096)
    assert c.train_batch_size == 64 and c.zero.reduce_bucket_size == 4096 ** 2
    assert c.zero.stage3_param_persistence_threshold == 40960
    with pytest.raises(ValueError):
        load_ds_config({"train_batch_size": 10, "train_micro_batch_size_per_gpu": 2,
                        "gradient_accumulation_steps": 1}, world_size=4)


def test_initialize_api():
    net = Net()
    opt = torch.optim.AdamW(net.parameters(), lr=3e-4, weight_decay=0.1)
    eng, o, _, sched = initialize(net, {"train_micro_batch_size_per_gpu": 4,
                                        "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0,
                                                                                     "warmup_max_lr": 3e-4,
                                                                                     "warmup_num_steps": 10}}},
                                  optimizer=opt)
    assert eng.lr == 3e-4 and eng.wd == 0.1 and sched is not None and eng.get_lr()[0] == 0.0


def _fsdp_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from llm_in_practise_amd.parallel.fsdp import FSDP, ShardingStrategy, get_state_dict, \
        transformer_auto_wrap_policy
    torch.manual_seed(0)
    net = Net()
    m = FSDP(net, auto_wrap_policy=transformer_auto_wrap_policy({nn.Sequential}),
             sharding_strategy=ShardingStrategy.FULL_SHARD, lr=1e-2, weight_decay=0.01, grad_clip=0.05)
    for s in range(3):
        x, y = _data(s, rank)
        m.backward(((m(x) - y) ** 2).mean())
        m.step()
    sd, _ = get_state_dict(m)
    if rank == 0:
        torch.save(sd, out)
    torch.distributed.destroy_process_group()


def test_fsdp_api_full_shard_matches_single_process(tmp_path):
    out = str(tmp_path / "f.pt")
    mp.spawn(_fsdp_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want = _oracle()
    for k in want:
        assert torch.allclose(got[k], want[k], atol=2e-5), k


# ----------------------------------------------------------------------------- stage-3 scheduling
def _cfg3(prefetch, reuse, bucket=64):
    c = _cfg(3)
    c["zero_optimization"].update({"stage3_prefetch_bucket_size": prefetch, "stage3_max_reuse_distance": reuse,
                                   "stage3_param_persistence_threshold": 0, "reduce_bucket_size": bucket,
                                   "overlap_comm": True, "stage3_max_live_parameters": 10 ** 9})
    return c


def _prefetch_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = Net(n=5)
    eng = ZeroEngine(net, _cfg3(prefetch=1, reuse=0))     # prefetch one unit ahead, free after every use
    for step in range(3):                                 # step 0 records the execution order
        eng.log_events = step > 0
        x, y = _data(step, rank)
        eng.backward(((eng(x) - y) ** 2).mean())
        eng.step()
    sd = eng.consolidated_state_dict()
    if rank == 0:
        torch.save({"log": eng.event_log, "order": eng.fwd_order, "sd": sd}, out)
    torch.distributed.destroy_process_group()


def test_stage3_prefetch_issues_gathers_ahead_of_use(tmp_path):
    """Every block's all-gather is issued (async) while an EARLIER unit runs — before its own
    forward / backward use — and training still matches the single-process oracle."""
    out = str(tmp_path / "p.pt")
    mp.spawn(_prefetch_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    log, order = [tuple(e) for e in r["log"]], r["order"]
    assert len(order) == 5
    ahead, prev_use = 0, None
    for pos, (what, u) in enumerate(log):
        if what not in ("use_fwd", "use_bwd"):
            continue
        # prefetched = its gather was issued after the previous unit's use began, before this use
        if prev_use is not None and ("issue", u) in log[prev_use:pos]:
            ahead += 1
        prev_use = pos
    # per step: blocks 2..5 prefetched in the forward, 4..1 in the backward (2 logged steps)
    assert ahead == 2 * (4 + 4), log
    want = _oracle(steps=3, n=5)
    for k in want:
        assert torch.allclose(r["sd"][k], want[k], atol=2e-5), k


def _repart_save(rank, world, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    for stage in (1, 3):
        torch.manual_seed(0)
        eng = ZeroEngine(Net(), _cfg(stage))
        _train(eng, world, rank, steps=2)
        eng.save_checkpoint(os.path.join(d, f"s{stage}"))
    torch.distributed.destroy_process_group()


def test_checkpoint_repartitions_across_world_sizes(tmp_path):
    """A ZeRO-1 / ZeRO-3 checkpoint written by 2 ranks resumes in 1 process: the next step on the
    concatenated batch equals the 2-rank oracle's third step."""
    d = str(tmp_path / "ck")
    mp.spawn(_repart_save, args=(2, _free_port(), d), nprocs=2, join=True)
    want = _oracle(steps=3)
    for stage in (1, 3):
        torch.manual_seed(7)
        eng = ZeroEngine(Net(), _cfg(stage))
        eng.load_checkpoint(os.path.join(d, f"s{stage}"))
        xs, ys = zip(*[_data(2, r) for r in range(2)])
        eng.backward(((eng(torch.cat(xs)) - torch.cat(ys)) ** 2).mean())
        eng.step()
        got = eng.consolidated_state_dict()
        for k in want:
            assert torch.allclose(got[k], want[k], atol=2e-5), (stage, k)


class CkptNet(Net):
    def forward(self, x):
        import torch.utils.checkpoint as ckpt
        h = self.inp(x)
        for b in self.blocks:
            h = h + ckpt.checkpoint(b, h, use_reentrant=True)
        return self.out(h)


def test_stage3_forward_order_recorded_under_reentrant_checkpointing():
    """the first forward of a reentrant-checkpointed model runs under no_grad; the
    prefetch order must still be the forward order (not the reversed recompute order), and the
    engine trains identically to the un-checkpointed model."""
    outs = []
    for cls in (CkptNet, Net):
        torch.manual_seed(0)
        net = cls(d=32, n=4)
        eng = ZeroEngine(net, {"zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 10},
                               "optimizer": {"type": "AdamW", "params": {"lr": 1e-2}}})
        blocks = [u.index for u in eng.units if u.module in list(net.blocks)]
        for s in range(3):
            x, y = _data(s, 0)
            x.requires_grad_(True)
            eng.backward(((eng(x) - y) ** 2).mean())
            eng.step()
            pos = [eng.fwd_order.index(i) for i in blocks]
            assert pos == sorted(pos), (cls.__name__, s, eng.fwd_order)
        outs.append(eng.consolidated_state_dict())
    for k in outs[1]:
        assert torch.allclose(outs[0][k], outs[1][k], atol=1e-6), k


# ----------------------------------------------------------------------------- ZeRO + client 8-bit AdamW
def _w8(rank, world, port, stage, out, steps=4, ckpt=None, load=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = Net(d=40, n=3)            # 40x40 blocks: units are not multiples of 256 (uneven padded shards)
    eng = ZeroEngine(net, _cfg(stage), optim="paged_adamw_8bit")
    start = 0
    if load:
        eng.load_checkpoint(load)
        start = eng.global_steps
        # the re-partitioned 8-bit moments' padding decodes to the zero code (no phantom moment)
        real = eng._shard_of(torch.ones(sum(eng._layout()), dtype=torch.uint8)).bool().to(eng.qm.device)
        if (~real).any():
            z_s = eng.code_s[torch.argmin(eng.code_s.abs())]
            z_u = eng.code_u[torch.argmin(eng.code_u.abs())]
            assert torch.all(eng.code_s[eng.qm.long()][~real] == z_s)
            assert torch.all(eng.code_u[eng.qv.long()][~real] == z_u)
    for s in range(start, start + steps):
        xs, ys = zip(*[_data(s, r) for r in range(4)])
        per = 8 // world            # the same global batch of 8 rows at every world size
        x = torch.cat(xs)[:8].view(world, per, 8)[rank]
        y = torch.cat(ys)[:8].view(world, per, 1)[rank]
        eng.backward(((eng(x) - y) ** 2).mean())
        eng.step()
    if ckpt:
        eng.save_checkpoint(ckpt)
    sd = eng.consolidated_state_dict()
    if rank == 0:
        torch.save({"sd": sd, "am": eng.am.clone(), "optim": eng.optim_name}, out)
    torch.distributed.destroy_process_group()


def _w8_oracle(steps=4, stage=0):
    """Single process, same 8-bit blocking: the flat layout (stages 0-2) or the per-unit layout (3)."""
    torch.manual_seed(0)
    net = Net(d=40, n=3)
    eng = ZeroEngine(net, _cfg(stage), optim="paged_adamw_8bit")
    for s in range(steps):
        xs, ys = zip(*[_data(s, r) for r in range(4)])
        eng.backward(((eng(torch.cat(xs)[:8]) - torch.cat(ys)[:8]) ** 2).mean())
        eng.step()
    return net.state_dict()


@pytest.mark.parametrize("stage,world", [(3, 2), (3, 4), (2, 4), (1, 2)])
def test_zero_with_client_8bit_adamw_matches_single_process(tmp_path, stage, world):
    """E6 (qwen3-14b-qlora-dist-deepspeed.py:151,164): optim=paged_adamw_8bit under ZeRO keeps
    blockwise-8-bit moments on each rank's partition; shards are whole 256-element blocks, so the
    update equals the single-process 8-bit update at world 2 and 4 (to fp32 reduction-order noise)."""
    out = str(tmp_path / "w8.pt")
    mp.spawn(_w8, args=(world, _free_port(), stage, out), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    assert got["optim"] == "paged_adamw_8bit"
    want = _w8_oracle(stage=3 if stage == 3 else 0)
    for k in want:
        assert torch.allclose(got["sd"][k], want[k], atol=1e-4), (stage, world, k, (got["sd"][k] - want[k]).abs().max())


def test_zero3_8bit_checkpoint_repartitions_4_to_2(tmp_path):
    """8-bit states in the zero_pp_rank_* shards, re-partitioned on load (world 4 -> 2): training
    resumed at world 2 equals uninterrupted training."""
    ck = str(tmp_path / "ck")
    mp.spawn(_w8, args=(4, _free_port(), 3, str(tmp_path / "a.pt"), 2, ck), nprocs=4, join=True)
    mp.spawn(_w8, args=(2, _free_port(), 3, str(tmp_path / "b.pt"), 2, None, ck), nprocs=2, join=True)
    resumed = torch.load(str(tmp_path / "b.pt"), weights_only=True)["sd"]
    want = _w8_oracle(steps=4, stage=3)
    for k in want:
        assert torch.allclose(resumed[k], want[k], atol=1e-4), (k, (resumed[k] - want[k]).abs().max())
