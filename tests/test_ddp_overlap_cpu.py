"""Flat-buffer DDP with backward overlap (gloo, world_size 2): bucket all-reduces are issued from
gradient-ready hooks DURING the backward, and the averaged gradients / trained weights equal the
single-process oracle on the concatenated batch (ddp_basics/ddp_gpt_wikitext2.py:274 semantics)."""
import os
import socket

import torch
import torch.multiprocessing as mp
import torch.nn as nn

from llm_in_practise_amd.optim.adamw import AdamW
from llm_in_practise_amd.parallel.ddp import DistributedDataParallel


class Net(nn.Module):
    def __init__(self, d=32, n=6):
        super().__init__()
        self.inp = nn.Linear(8, d)
        self.blocks = nn.ModuleList([nn.Linear(d, d) for _ in range(n)])
        self.out = nn.Linear(d, 1)

    def forward(self, x):
        h = self.inp(x)
        for b in self.blocks:
            h = h + torch.tanh(b(h))
        return self.out(h)


def _data(step, rank, n=4):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(n, 8, generator=g), torch.randn(n, 1, generator=g)


def _worker(rank, world, port, out, ga, car=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = Net()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    ddp = DistributedDataParallel(net, flat=opt.flat, bucket_mb=0.004,   # ~1k floats: several buckets
                                  custom_allreduce="auto-host" if car else None)
    logs = []
    for s in range(3):
        for m in range(ga):
            x, y = _data(s * ga + m, rank)
            ctx = ddp.no_sync() if m < ga - 1 else torch.enable_grad()
            with ctx:
                ((ddp(x) - y) ** 2).mean().div(ga).backward()
        logs.append(list(ddp.launch_log))
        ddp.reset_log()
        ddp.allreduce_grads()
        opt.step()
        opt.zero_grad()
    calls = dict(ddp.car.calls) if ddp.car is not None else {}
    if ddp.car is not None:
        ddp.car.close()
    if rank == 0:
        torch.save({"sd": net.state_dict(), "logs": logs, "nb": len(ddp._buckets), "calls": calls}, out)
    torch.distributed.destroy_process_group()


def _oracle(ga):
    torch.manual_seed(0)
    net = Net()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    for s in range(3):
        for m in range(ga):
            xs, ys = zip(*[_data(s * ga + m, r) for r in range(2)])
            ((net(torch.cat(xs)) - torch.cat(ys)) ** 2).mean().div(ga).backward()
        opt.step()
        opt.zero_grad()
    return net.state_dict()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_overlap_matches_oracle_and_launches_during_backward(tmp_path):
    for ga in (1, 2):
        out = str(tmp_path / f"r{ga}.pt")
        mp.spawn(_worker, args=(2, _port(), out, ga), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)
        want = _oracle(ga)
        for k in want:
            assert torch.allclose(got["sd"][k], want[k], atol=1e-5), k
        assert got["nb"] >= 3
        for log in got["logs"]:
            # every bucket was issued from a gradient-ready hook inside backward, in reverse order
            assert [why for _, why in log] == ["hook"] * got["nb"]
            assert [b for b, _ in log] == list(range(got["nb"]))


def test_ddp_buckets_over_custom_allreduce_match_oracle(tmp_path):
    """Gradient buckets through the peer-memory all-reduce (its /dev/shm model on CPU)."""
    out = str(tmp_path / "car.pt")
    mp.spawn(_worker, args=(2, _port(), out, 2, True), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want = _oracle(2)
    for k in want:
        assert torch.allclose(got["sd"][k], want[k], atol=1e-5), k
    assert got["calls"]["oneshot"] + got["calls"]["twoshot"] > 0


class SkipNet(Net):
    """A block that one rank never runs (an MoE expert that got zero tokens on that rank)."""

    def forward(self, x, skip=None):
        h = self.inp(x)
        for i, b in enumerate(self.blocks):
            if i != skip:
                h = h + torch.tanh(b(h))
        return self.out(h)


def _skip_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = SkipNet()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    ddp = DistributedDataParallel(net, flat=opt.flat, bucket_mb=0.004)
    logs = []
    for s in range(3):
        x, y = _data(s, rank)
        # the last block (the FIRST bucket in backward order) is unused on rank 1
        ((ddp(x, skip=5 if rank == 1 else None) - y) ** 2).mean().backward()
        logs.append(list(ddp.launch_log))
        ddp.reset_log()
        ddp.allreduce_grads()
        logs[-1] += list(ddp.launch_log)
        ddp.reset_log()
        opt.step()
        opt.zero_grad()
    torch.save({"sd": net.state_dict(), "logs": logs, "nb": len(ddp._buckets)}, out.format(rank))
    torch.distributed.destroy_process_group()


def test_ddp_unused_param_on_one_rank_keeps_collective_order(tmp_path):
    """with a parameter unused on one rank, buckets must still be issued in the same
    (index) order on every rank; gradients equal the per-rank-average oracle."""
    out = str(tmp_path / "skip{}.pt")
    mp.spawn(_skip_worker, args=(2, _port(), out), nprocs=2, join=True)
    torch.manual_seed(0)
    net = SkipNet()
    opt = AdamW(net.parameters(), lr=1e-2, weight_decay=0.0)
    for s in range(3):
        loss = sum(((net(_data(s, r)[0], skip=5 if r == 1 else None) - _data(s, r)[1]) ** 2).mean() for r in range(2))
        (loss / 2).backward()
        opt.step()
        opt.zero_grad()
    for r in range(2):
        got = torch.load(out.format(r), weights_only=True)
        for k, v in net.state_dict().items():
            assert torch.allclose(got["sd"][k], v, atol=1e-5), (r, k)
        for log in got["logs"]:
            assert [b for b, _ in log] == list(range(got["nb"]))      # identical order on both ranks
        if r == 1:   # the unused block holds back its bucket and everything after it until the flush
            assert all(log[0][1] == "flush" for log in got["logs"])
