"""Aux subsystems: collective-sequence checker, fault injector, metrics, timer."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llm_in_practise_amd.parallel.checker import CollectiveChecker, CollectiveMismatch
from llm_in_practise_amd.utils.faults import FaultInjector, InjectedFault
from llm_in_practise_amd.utils.metrics import MetricsWriter, read_jsonl
from llm_in_practise_amd.utils.timer import StepTimer


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _barrier_bug_worker(rank, world, port, out):
    """Reproduces temp/ddp_gpt_bpe_tokenizer.py:369-387: rank 0 runs one barrier, others two."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = "ok"
    try:
        with CollectiveChecker(every=1):
            dist.barrier()
            if rank != 0:
                dist.barrier()
            t = torch.zeros(4)
            dist.broadcast(t, 0)
    except CollectiveMismatch as e:
        res = "mismatch"
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_checker_flags_rank0_only_barrier(tmp_path):
    out = str(tmp_path / "r")
    mp.spawn(_barrier_bug_worker, args=(2, _port(), out), nprocs=2, join=True)
    assert torch.load(out + ".0") == "mismatch" and torch.load(out + ".1") == "mismatch"


def _clean_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with CollectiveChecker(every=1) as c:
        t = torch.ones(3) * rank
        dist.all_reduce(t)
        dist.barrier()
    torch.save((c.seq, float(t[0])), f"{out}.{rank}")
    dist.destroy_process_group()


def test_checker_passes_matching_sequences(tmp_path):
    out = str(tmp_path / "r")
    mp.spawn(_clean_worker, args=(2, _port(), out), nprocs=2, join=True)
    assert torch.load(out + ".0") == (2, 1.0)


def test_fault_injector():
    f = FaultInjector("0:3:raise,*:5:nan,1:2:raise", rank=0)
    assert f.check(2) is None
    with pytest.raises(InjectedFault):
        f.check(3)
    assert f.check(3) is None                    # fires once
    assert f.check(5) == "nan"
    assert not FaultInjector("", rank=0)


def test_metrics_and_timer(tmp_path):
    p = str(tmp_path / "m.jsonl")
    w = MetricsWriter(p)
    w.write(step=1, loss=2.0)
    w.write(step=2, loss=1.5)
    w.close()
    r = read_jsonl(p)
    assert [x["step"] for x in r] == [1, 2] and r[1]["loss"] == 1.5
    t = StepTimer()
    with t.phase("a"):
        sum(range(1000))
    s = t.summary()
    assert "a" in s and s["a"] >= 0


def _hc_worker(rank, world, port, q):
    import os as _os
    import torch as _t
    _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _t.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from llm_in_practise_amd.parallel.healthcheck import cluster_check
    q.put((rank, cluster_check(allreduce_mib=1, iters=1)))
    _t.distributed.destroy_process_group()


def test_cluster_check_gloo():
    """H4 health probe: inventory of every rank, broadcast + all-reduce values verified."""
    import socket as _s
    import torch.multiprocessing as _mp
    s = _s.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = _mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_hc_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    assert res[1] is None
    rep = res[0]
    assert rep["all_ok"] and rep["world_size"] == 2 and len(rep["ranks"]) == 2
