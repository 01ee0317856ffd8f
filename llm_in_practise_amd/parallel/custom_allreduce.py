"""Intra-node custom all-reduce over xGMI peer memory.

The reference toggles vLLM's custom all-reduce for single-node tensor parallelism
(``Quantization/LLM-Compressor/AWQ/eval_qwen3_4b_awq.py:20``).  On MI355X the 8 GPUs of a node
form a full xGMI mesh, so every GPU can load from every peer's HBM through IPC-mapped pointers;
for the latency-bound buffers of LoRA fine-tuning (a few MB of adapter gradients, norm partials,
TP activations of a decode step) that beats a ring collective, which pays 2·(W−1) dependent hops.

Design (kernel: ``csrc/kernels/allreduce.hip``):

* ONE registry per process group, built once: every rank allocates a staging area
  ``data[2][cap] | result[2][cap]`` and an uncached flag array ``uint32 flags[2][8][64]``, exports
  IPC handles, and opens every peer's (``hipIpcOpenMemHandle``) — a call never allocates or maps.
* Algorithm by size: one-shot (every rank reads all W inputs, one cross-GPU barrier) up to
  ``one_shot_bytes``; two-shot (rank r reduces slice r, barrier, everyone gathers the reduced
  slices) up to ``max_bytes``; larger buffers — and anything not eligible (CPU tensors, other
  dtypes, unaligned sizes, multi-node groups) — fall back to RCCL through ``torch.distributed``.
* Epoch-stamped flags (never reset) + staging double-buffered on epoch parity, so back-to-back
  calls need no trailing barrier (argument in the kernel header).
* The protocol is backend-independent: :class:`_HostPeers` runs the SAME layout, epochs, parity
  and barriers over ``/dev/shm`` files with a Python "kernel", which is what the CPU multi-process
  tests exercise; :class:`_HipPeers` maps it onto IPC memory and the HIP kernel.

``LIPA_CUSTOM_AR=1`` makes :class:`~.ddp.DistributedDataParallel` build one for its gradient
buckets (``custom_allreduce="auto"``); default off until it is measured on an 8-GPU node.
"""
from __future__ import annotations

import os
import time
import uuid

import numpy as np
import torch
import torch.distributed as dist

NBAR, MAXW, MAXB = 2, 8, 64
FLAG_WORDS = NBAR * MAXW * MAXB


def choose_algorithm(nbytes: int, world: int, one_shot_bytes: int, max_bytes: int,
                     one_shot_w2: bool = True) -> str | None:
    """'oneshot' | 'twoshot' | None (use RCCL)."""
    if world < 2 or world > MAXW or nbytes == 0 or nbytes % 16 or nbytes > max_bytes:
        return None
    if (world == 2 and one_shot_w2) or nbytes <= one_shot_bytes:   # W = 2: same traffic, one barrier fewer
        return "oneshot"
    return "twoshot"


class _HostPeers:
    """CPU model of the peer-memory protocol: each rank's staging + flags in a ``/dev/shm`` file
    mapped by every rank (x86 stores are seen in program order, like release/acquire here)."""

    def __init__(self, token: str, rank: int, world: int, cap: int):
        self.rank, self.world, self.cap = rank, world, cap
        self.size = FLAG_WORDS * 4 + 4 * cap
        self.path = f"/dev/shm/lipa_car_{token}_{rank}"
        with open(self.path, "wb") as f:
            f.truncate(self.size)
        self.maps: list[np.memmap] = []

    def open_peers(self, token: str):
        self.maps = [np.memmap(f"/dev/shm/lipa_car_{token}_{p}", dtype=np.uint8, mode="r+", shape=(self.size,))
                     for p in range(self.world)]

    def flags(self, p: int) -> np.ndarray:
        return self.maps[p][:FLAG_WORDS * 4].view(np.uint32).reshape(NBAR, MAXW, MAXB)

    def region(self, p: int, which: str, parity: int) -> np.ndarray:
        base = FLAG_WORDS * 4 + (0 if which == "data" else 2 * self.cap) + parity * self.cap
        return self.maps[p][base:base + self.cap]

    def barrier(self, k: int, epoch: int, timeout: float = 60.0):
        for p in range(self.world):
            self.flags(p)[k, self.rank, 0] = epoch
        mine = self.flags(self.rank)
        t0 = time.monotonic()
        while (mine[k, :self.world, 0] < epoch).any():
            if time.monotonic() - t0 > timeout:
                raise RuntimeError(f"custom all-reduce: peer missed barrier {k} of epoch {epoch}")
            time.sleep(0)

    def all_reduce(self, t: torch.Tensor, epoch: int, two_shot: bool, scale: float):
        par = epoch & 1
        nbytes = t.numel() * t.element_size()
        src = t.detach().contiguous().view(torch.uint8).numpy()
        self.region(self.rank, "data", par)[:nbytes] = src
        self.barrier(0, epoch)
        tdt = t.dtype

        def peer_vals(p, lo, hi, which="data"):
            raw = torch.from_numpy(np.array(self.region(p, which, par)[lo:hi]))
            return raw.view(tdt).float()

        W = self.world
        if not two_shot:
            acc = sum(peer_vals((self.rank + j) % W, 0, nbytes) for j in range(W))
            t.copy_((acc * scale).to(tdt).view(t.shape))
            return
        nvec = nbytes // 16
        per = (nvec + W - 1) // W
        s0, s1 = min(nvec, per * self.rank) * 16, min(nvec, per * (self.rank + 1)) * 16
        if s1 > s0:
            acc = sum(peer_vals((self.rank + j) % W, s0, s1) for j in range(W))
            self.region(self.rank, "result", par)[:s1 - s0] = (acc * scale).to(tdt).view(torch.uint8).numpy()
        self.barrier(1, epoch)
        out = bytearray(nbytes)
        for owner in range(W):
            o0, o1 = min(nvec, per * owner) * 16, min(nvec, per * (owner + 1)) * 16
            if o1 > o0:
                out[o0:o1] = bytes(self.region(owner, "result", par)[:o1 - o0])
        t.copy_(torch.frombuffer(out, dtype=torch.uint8).view(tdt).view(t.shape))

    def close(self):
        self.maps = []
        try:
            os.unlink(self.path)
        except FileNotFoundError:
            pass


class _HipPeers:
    """IPC-mapped staging + flags on the GPUs, the reduction in ``allreduce.hip``."""

    def __init__(self, rank: int, world: int, cap: int, device: torch.device):
        from ..ops._native import native
        self.nat = native()
        self.rank, self.world, self.cap = rank, world, cap
        with torch.cuda.device(device):
            self.stage = self.nat.car_alloc(4 * cap, False)              # data[2] | result[2]
            self.flag = self.nat.car_alloc(FLAG_WORDS * 4, True)         # uncached: polled across GPUs
            self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.handles = (self.nat.car_handle(self.stage), self.nat.car_handle(self.flag))
        self.peer_stage: list[int] = []
        self.peer_flag: list[int] = []
        self.opened: list[int] = []

    def open_peers(self, all_handles):
        for p, (hs, hf) in enumerate(all_handles):
            if p == self.rank:
                self.peer_stage.append(self.stage)
                self.peer_flag.append(self.flag)
            else:
                s, f = self.nat.car_open(hs), self.nat.car_open(hf)
                self.opened += [s, f]
                self.peer_stage.append(s)
                self.peer_flag.append(f)

    def all_reduce(self, t: torch.Tensor, epoch: int, two_shot: bool, scale: float, blocks: int):
        par = epoch & 1
        data = [s + par * self.cap for s in self.peer_stage]
        res = [s + (2 + par) * self.cap for s in self.peer_stage]
        self.nat.custom_allreduce(t, data, res, self.peer_flag, self.err, self.rank, epoch, two_shot, scale, blocks)

    def check(self):
        if int(self.err.item()):
            raise RuntimeError("custom all-reduce: a peer missed a barrier (timeout inside the kernel)")

    def close(self):
        for p in self.opened:
            self.nat.car_close(p)
        self.nat.car_free(self.stage)
        self.nat.car_free(self.flag)
        self.opened = []


class CustomAllReduce:
    """One-shot / two-shot peer-memory all-reduce for one intra-node process group, RCCL fallback.

    ``backend``: "hip" (IPC + kernel), "host" (the /dev/shm model — CPU tensors), "auto" (hip for
    a CUDA ``device``, host otherwise)."""

    def __init__(self, group=None, max_bytes: int = 8 << 20, one_shot_bytes: int = 256 << 10,
                 backend: str = "auto", device=None, blocks: int = 32, one_shot_w2: bool = True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.max_bytes = (max_bytes + 15) // 16 * 16
        self.one_shot_bytes = one_shot_bytes
        self.blocks = min(blocks, MAXB)
        self.one_shot_w2 = one_shot_w2
        self.epoch = 0
        self.calls = {"oneshot": 0, "twoshot": 0, "fallback": 0}
        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        if backend == "auto":
            backend = "hip" if dev.type == "cuda" else "host"
        self.backend, self.device = backend, dev
        hosts: list = [None] * self.world
        dist.all_gather_object(hosts, os.uname().nodename, group=group)
        self.enabled = len(set(hosts)) == 1 and 2 <= self.world <= MAXW
        self.peers = None
        if not self.enabled:
            return
        if backend == "host":
            tok = [uuid.uuid4().hex if self.rank == 0 else None]
            dist.broadcast_object_list(tok, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            self.peers = _HostPeers(tok[0], self.rank, self.world, self.max_bytes)
            dist.barrier(group=group)
            self.peers.open_peers(tok[0])
            dist.barrier(group=group)
        else:
            self.peers = _HipPeers(self.rank, self.world, self.max_bytes, dev)
            allh: list = [None] * self.world
            dist.all_gather_object(allh, self.peers.handles, group=group)
            self.peers.open_peers(allh)
            torch.cuda.synchronize(dev)
            dist.barrier(group=group)

    # ------------------------------------------------------------------ dispatch
    def algorithm(self, t: torch.Tensor) -> str | None:
        if not self.enabled or not t.is_contiguous() or t.dtype not in (torch.float32, torch.bfloat16):
            return None
        if (self.backend == "hip") != t.is_cuda:
            return None
        if t.is_cuda and t.data_ptr() % 16:
            return None
        return choose_algorithm(t.numel() * t.element_size(), self.world, self.one_shot_bytes, self.max_bytes,
                                self.one_shot_w2)

    def should_use(self, t: torch.Tensor) -> bool:
        return self.algorithm(t) is not None

    def all_reduce_(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In-place sum (or mean) over the group; RCCL/gloo when the peer path does not apply."""
        algo = self.algorithm(t)
        if algo is None:
            self.calls["fallback"] += 1
            dist.all_reduce(t, group=self.group)
            if average:
                t.div_(self.world)
            return t
        self.epoch += 1
        self.calls[algo] += 1
        scale = 1.0 / self.world if average else 1.0
        if self.backend == "host":
            self.peers.all_reduce(t, self.epoch, algo == "twoshot", scale)
        else:
            self.peers.all_reduce(t, self.epoch, algo == "twoshot", scale, self.blocks)
        return t

    def check(self):
        """Raise if a kernel-side barrier timed out (syncs the device; call off the hot path)."""
        if self.backend == "hip" and self.peers is not None:
            self.peers.check()

    def poll(self):
        """Off-the-hot-path timeout check, once per optimizer step (DDP calls it after joining the
        gradient buckets): the device error word copied at the PREVIOUS call — long finished by now —
        is examined, then a fresh non-blocking copy is queued behind this step's reductions.  A
        kernel-side barrier timeout (a peer that never arrived: its staging was stale) therefore
        raises at the next step boundary instead of letting training continue on corrupted
        gradients; the word is reset so a caller that handles the error can go on."""
        peers = self.peers
        if self.backend != "hip" or peers is None:
            return
        err = peers.err
        pend = getattr(peers, "pending", None)
        if pend is not None:
            ev, host = pend
            if ev is not None:
                ev.synchronize()
            if int(host[0]):
                peers.pending = None
                err.zero_()
                raise RuntimeError("custom all-reduce: a peer missed a kernel-side barrier (timeout); "
                                   "the reduced gradients of that step are not valid")
        host = getattr(peers, "host_err", None)
        if host is None:
            host = peers.host_err = torch.zeros(1, dtype=torch.int32, pin_memory=err.is_cuda)
        host.copy_(err, non_blocking=err.is_cuda)
        ev = None
        if err.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        peers.pending = (ev, host)

    def close(self):
        if self.peers is not None:
            if self.backend == "hip":
                torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)      # nobody may still read a peer's staging
            self.peers.close()
            self.peers = None
            self.enabled = False
