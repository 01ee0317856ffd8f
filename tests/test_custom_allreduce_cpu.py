"""Custom all-reduce protocol (parallel/custom_allreduce.py) on CPU: the /dev/shm model of the
IPC peer-memory layout runs the same epochs / parity / barriers as the HIP kernel; gloo carries
the handle exchange and the RCCL-fallback path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llm_in_practise_amd.parallel.custom_allreduce import choose_algorithm


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_choose_algorithm_thresholds():
    assert choose_algorithm(1024, 8, 4096, 1 << 20) == "oneshot"
    assert choose_algorithm(8192, 8, 4096, 1 << 20) == "twoshot"
    assert choose_algorithm(8192, 2, 4096, 1 << 20) == "oneshot"      # W=2: one barrier fewer
    assert choose_algorithm(2 << 20, 8, 4096, 1 << 20) is None         # above the staging cap -> RCCL
    assert choose_algorithm(1000, 8, 4096, 1 << 20) is None            # not a multiple of 16 B
    assert choose_algorithm(1024, 1, 4096, 1 << 20) is None
    assert choose_algorithm(1024, 9, 4096, 1 << 20) is None


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llm_in_practise_amd.parallel.custom_allreduce import CustomAllReduce
    car = CustomAllReduce(max_bytes=64 << 10, one_shot_bytes=4 << 10, backend="host")
    ok = []
    try:
        for step, (n, dt) in enumerate([(256, torch.float32), (8192, torch.float32), (4096, torch.bfloat16),
                                        (24 << 10, torch.float32), (8, torch.float32), (8192, torch.bfloat16)] * 2):
            g = torch.Generator().manual_seed(1000 * step + rank)
            t = torch.randn(n, generator=g).to(dt)
            ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(1000 * step + r)).to(dt).float()
                      for r in range(world))
            avg = step % 2 == 1
            car.all_reduce_(t, average=avg)
            want = ref / world if avg else ref
            tol = 2e-2 if dt == torch.bfloat16 else 1e-5
            ok.append(bool(torch.allclose(t.float(), want, rtol=tol, atol=tol * 4)))
        out_q.put((rank, ok, dict(car.calls)))
    finally:
        car.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_protocol_matches_sum(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, ok, calls in res:
        assert all(ok), (rank, ok)
        # 256 floats (1 KB) and 8 floats one-shot; 32 KB and 8 KB bf16 two-shot (W>2); 96 KB > cap -> fallback
        assert calls["fallback"] == 2
        if world == 2:
            assert calls["oneshot"] == 10 and calls["twoshot"] == 0
        else:
            assert calls["oneshot"] == 4 and calls["twoshot"] == 6
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("lipa_car_")]


def test_poll_raises_on_kernel_timeout_word_and_resets():
    """the kernel's timeout word is checked off the hot path (one step later) and reset."""
    import types

    import pytest
    import torch

    from llm_in_practise_amd.parallel.custom_allreduce import CustomAllReduce
    car = CustomAllReduce.__new__(CustomAllReduce)
    car.backend = "hip"
    car.peers = types.SimpleNamespace(err=torch.zeros(1, dtype=torch.int32))
    car.poll()                      # queues a copy of a clean word
    car.poll()                      # clean -> no error
    car.peers.err[0] = 1            # a kernel-side barrier timed out during this step
    car.poll()                      # examines the previous (clean) copy, queues this one
    with pytest.raises(RuntimeError, match="missed a kernel-side barrier"):
        car.poll()
    assert int(car.peers.err[0]) == 0
    car.poll()
    car.poll()
