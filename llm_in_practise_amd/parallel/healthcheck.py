"""Cluster health check over ``torch.distributed`` (``ray_cluster_healthcheck.py``
probes nodes / CPUs / GPUs and fans a 2048² array out through the object store; the NCCL env
knobs of ``Fine-Tuning/README.md:254-262`` are the usual bring-up suspects).

Run under torchrun on every node (``lipa cluster-check``): each rank reports host, device and
HBM; rank 0 prints the inventory, then times a broadcast of a 2048×2048 fp32 array (the
reference's fan-out payload) and a bucket-sized all-reduce, and checks the reduced values —
a wrong sum or a hang pinpoints the bad link / rank before a training job finds it.
"""
from __future__ import annotations

import os
import socket
import time

import torch
import torch.distributed as dist


def _device_info() -> dict:
    info = {"host": socket.gethostname(), "pid": os.getpid(), "cpus": os.cpu_count()}
    if torch.cuda.is_available():
        i = torch.cuda.current_device()
        p = torch.cuda.get_device_properties(i)
        info.update(device=f"cuda:{i}", name=p.name, arch=getattr(p, "gcnArchName", ""), hbm_gib=round(
            p.total_memory / 2 ** 30, 1), cus=p.multi_processor_count)
    else:
        info.update(device="cpu")
    for k in ("NCCL_SOCKET_IFNAME", "NCCL_IB_DISABLE", "NCCL_P2P_DISABLE", "HSA_ENABLE_IPC_MODE_LEGACY"):
        if k in os.environ:
            info[k] = os.environ[k]
    return info


def _timed(fn, iters: int) -> float:
    fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def cluster_check(allreduce_mib: int = 64, iters: int = 5) -> dict | None:
    """Collective probe; returns the report on rank 0 (None elsewhere)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    infos = [None] * world
    dist.all_gather_object(infos, _device_info())
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    arr = torch.full((2048, 2048), float(rank == 0), device=dev)
    dist.broadcast(arr, src=0)
    bcast_ok = bool((arr == 1).all())
    t_b = _timed(lambda: dist.broadcast(arr, src=0), iters)
    n = allreduce_mib * 2 ** 20 // 4
    buf = torch.full((n,), float(rank + 1), device=dev)
    dist.all_reduce(buf)
    ar_ok = bool(torch.allclose(buf[:4], torch.full((4,), world * (world + 1) / 2, device=dev)))
    t_ar = _timed(lambda: dist.all_reduce(buf), iters)
    flags = torch.tensor([int(bcast_ok and ar_ok)], device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank != 0:
        return None
    nbytes = n * 4
    return {"world_size": world, "backend": dist.get_backend(), "ranks": infos, "all_ok": bool(flags.item()),
            "broadcast_2048x2048_ms": round(t_b * 1e3, 3),
            "allreduce_MiB": allreduce_mib, "allreduce_ms": round(t_ar * 1e3, 3),
            # ring all-reduce moves 2(w-1)/w of the buffer per rank: the NCCL-tests "bus bandwidth"
            "allreduce_busbw_GBs": round(2 * (world - 1) / world * nbytes / t_ar / 1e9, 2)}
