"""Data parallel: ``DDP(model, device_ids=[local_rank])`` semantics
(``LLM_Distributed_Trainning/PyTorch/ddp_basics/ddp_gpt_wikitext2.py:274``).

MI355X design: gradients live in ONE flat fp32 buffer (owned by the fused optimizer, see
``optim/adamw.py``), so the data-parallel reduction is bucketed over that buffer and never
packs/unpacks.  Buckets are contiguous ranges of the flat buffer cut at parameter boundaries
in REVERSE parameter order (the order backward produces gradients).

Overlap with the backward: every parameter reports "gradient final" — through a
``post_accumulate_grad_hook`` for ordinary autograd leaves, and through
:func:`ops.linear.register_grad_ready` for the LoRA adapters whose gradients the fused
kernels accumulate in place — and once a bucket's last parameter has reported AND every bucket
before it has been issued, the bucket's all-reduce is issued on a side HIP stream (ordered
after the producing kernels by an event), so RCCL over xGMI runs while the GPU computes the rest
of the backward.  Buckets are issued strictly in index order (torch DDP's rule): collectives pair
up by call order, so a bucket that completes early on one rank must not overtake a bucket whose
parameter got no gradient on that rank (an MoE expert that received zero tokens) — it waits, and
``allreduce_grads()`` (after the boundary micro-step's backward) flushes the unfinished tail in
the same order on every rank, then joins the streams.  ``no_sync()`` skips the reduction on non-boundary
gradient-accumulation micro-steps.

Bucket size: xGMI rings are per-link bandwidth-bound, so buckets are large (default 32 MiB,
never fewer than ~4 per model so the first can start early); LoRA-sized gradient sets
(15-60 MB) become a few collectives.

Small buckets can go over the intra-node peer-memory all-reduce instead of RCCL
(``custom_allreduce=`` a :class:`~.custom_allreduce.CustomAllReduce`, or ``"auto"`` /
``LIPA_CUSTOM_AR=1`` to build one; default off until an 8-GPU run records it): one- or two-shot by
size, RCCL above its staging cap.

On start the module's parameters and buffers are broadcast from rank 0
(``sync_module_states``).
"""
from __future__ import annotations

import contextlib
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import COMM, all_reduce_mean_, is_dist


ONE_SHOT_BYTES = 256 << 10


def allreduce_path(nbytes: int, world: int, single_node: bool) -> str:
    """The gradient-bucket all-reduce decision, by message size:

    * ``"peer-oneshot"`` — one node, ≤ 256 KiB (a multiple of 16 B): latency-bound; every rank reads the
      W inputs once from IPC-mapped peer HBM over the xGMI mesh and one cross-GPU barrier ends it
      (parallel/custom_allreduce.py + csrc/kernels/allreduce.hip), instead of a ring's 2·(W−1)
      dependent hops;
    * ``"rccl"`` — everything else: bandwidth-bound buckets (the QLoRA adapter gradients are 15 MB
      for Qwen3-8B r8 q/v, bucketed ≥ 1 MiB) go to RCCL's ring / tree over the 7 xGMI links per GPU,
      which the peer two-shot does not beat by more than the ring's latency at these sizes;
    * ``"none"`` — a single rank."""
    if world < 2:
        return "none"
    if single_node and 0 < nbytes <= ONE_SHOT_BYTES and nbytes % 16 == 0:
        return "peer-oneshot"
    return "rccl"


class _Bucket:
    __slots__ = ("start", "end", "params", "remaining", "launched")

    def __init__(self, start: int, end: int, params: list[int]):
        self.start, self.end, self.params = start, end, params
        self.remaining = len(params)
        self.launched = False


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, grad_buffer: torch.Tensor | None = None, bucket_mb: float | None = None,
                 broadcast_buffers: bool = True, device_ids=None, find_unused_parameters: bool = False,
                 overlap: bool = True, flat=None, custom_allreduce=None, **_):
        super().__init__()
        self.module = module
        self.flat = flat
        self.grad_buffer = flat.grad if flat is not None else grad_buffer
        self._sync = True
        self.launch_log: list[tuple[int, str]] = []      # (bucket, "hook" | "flush") for the last step
        if is_dist():
            with torch.no_grad():
                for t in list(module.parameters()) + (list(module.buffers()) if broadcast_buffers else []):
                    dist.broadcast(t.data, src=0)
        self.overlap = overlap and flat is not None and is_dist()
        self._cuda = self.grad_buffer is not None and self.grad_buffer.is_cuda
        self._stream = torch.cuda.Stream(device=self.grad_buffer.device) if (self.overlap and self._cuda) else None
        self._works: list = []
        if custom_allreduce is None:
            # default off: the peer-memory path has no multi-GPU hardware record yet (parallel/custom_allreduce.py)
            custom_allreduce = os.environ.get("LIPA_CUSTOM_AR", "0")
            custom_allreduce = {"0": None, "off": None, "1": "auto"}.get(custom_allreduce, custom_allreduce)
        if self.grad_buffer is not None:
            total = self.grad_buffer.numel()
            cap = int((bucket_mb if bucket_mb is not None else 32.0) * (1 << 20) / 4)
            if bucket_mb is None:
                cap = max(1 << 20, min(cap, total // 4))
            self.bucket_elems = max(1, cap)
        if self.overlap:
            self._build_buckets()
        host_ok = custom_allreduce == "auto-host"     # the /dev/shm model of the protocol (CPU rehearsal)
        if custom_allreduce in ("auto", "auto-host") and not self.overlap:
            custom_allreduce = None         # the non-overlapped path reduces whole buckets on RCCL only
        if custom_allreduce == "auto-host" or (custom_allreduce == "auto" and self._cuda):
            # the decided policy (allreduce_path): a peer-memory one-shot all-reduce only for buckets that
            # are latency-bound (<= 256 KiB on one node); everything larger goes to RCCL.  Built only when
            # some bucket qualifies — the QLoRA headline's adapter-gradient buckets (≥ 1 MiB) never do,
            # so its multi-GPU step is plain RCCL
            custom_allreduce = None
            if is_dist() and self.grad_buffer is not None and (self._cuda or host_ok) and any(
                    allreduce_path(v.numel() * v.element_size(), dist.get_world_size(), True) != "rccl"
                    for v in self.buckets()):
                from .custom_allreduce import CustomAllReduce
                custom_allreduce = CustomAllReduce(device=self.grad_buffer.device, max_bytes=ONE_SHOT_BYTES,
                                                   one_shot_bytes=ONE_SHOT_BYTES)
        elif custom_allreduce == "auto":
            custom_allreduce = None
        self.car = custom_allreduce
        if self.overlap:
            self._hooks = []
            from ..ops.linear import register_grad_ready
            self._listener = register_grad_ready(self._on_ready)
            for p in flat.params:
                if hasattr(p, "register_post_accumulate_grad_hook"):
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulated))

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self):
        fp = self.flat
        order = sorted(range(len(fp.params)), key=lambda i: fp.offsets[i], reverse=True)
        self._bucket_of: dict[int, int] = {}
        self._index = {id(p): i for i, p in enumerate(fp.params)}
        self._buckets: list[_Bucket] = []
        end = fp.numel
        cur: list[int] = []
        for i in order:
            cur.append(i)
            start = fp.offsets[i]
            if end - start >= self.bucket_elems:
                self._buckets.append(_Bucket(start, end, cur))
                end, cur = start, []
        if cur and self._buckets and end < self.bucket_elems // 4:
            # a small remainder joins the previous bucket (one fewer latency-bound collective)
            self._buckets[-1].start = 0
            self._buckets[-1].params += cur
            self._buckets[-1].remaining = len(self._buckets[-1].params)
        elif cur:
            self._buckets.append(_Bucket(0, end, cur))
        elif self._buckets:
            self._buckets[-1].start = 0
        for b, bk in enumerate(self._buckets):
            for i in bk.params:
                self._bucket_of[i] = b
        self._ready = [False] * len(fp.params)
        self._next = 0          # the next bucket index allowed to launch (strict index order)

    def buckets(self) -> list[torch.Tensor]:
        g = self.grad_buffer
        if self.overlap:
            return [g[b.start:b.end] for b in self._buckets]
        return [g[s:s + self.bucket_elems] for s in range(0, g.numel(), self.bucket_elems)]

    def _launch(self, b: int, why: str):
        bk = self._buckets[b]
        if bk.launched:
            return
        bk.launched = True
        self.launch_log.append((b, why))
        view = self.grad_buffer[bk.start:bk.end]
        COMM.issue("all_reduce", view.numel() * view.element_size())
        if self._stream is not None:
            self._stream.wait_stream(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(self._stream):
                ev0 = COMM.events(self._stream)
                if self.car is not None and self.car.should_use(view):
                    self.car.all_reduce_(view, average=True)
                else:
                    all_reduce_mean_(view)
                COMM.span_end("all_reduce", ev0, self._stream)
        elif self.car is not None and self.car.should_use(view):     # peer-memory path (host model on CPU)
            self.car.all_reduce_(view, average=True)
        else:       # gloo / CPU: an async collective on the process group's own thread
            self._works.append((dist.all_reduce(view, async_op=True), view))

    def _mark(self, i: int):
        if not self._sync or self._ready[i]:
            return
        self._ready[i] = True
        b = self._bucket_of[i]
        bk = self._buckets[b]
        bk.remaining -= 1
        # issue every complete bucket at the head of the order; a complete bucket behind an
        # incomplete one waits (collectives must be called in the same order on every rank)
        while self._next < len(self._buckets) and self._buckets[self._next].remaining == 0:
            self._launch(self._next, "hook")
            self._next += 1

    def _on_accumulated(self, p: torch.Tensor):
        i = self._index.get(id(p))
        if i is None or not self._sync:
            return
        o = self.flat.offsets[i]
        if p.grad is not None and p.grad.data_ptr() != self.flat.grad_ptrs[i]:
            # low-precision parameter: fold its separately allocated grad into the flat buffer now
            self.flat.grad[o:o + p.numel()].add_(p.grad.reshape(-1).float())
            p.grad = None
        self._mark(i)

    def _on_ready(self, p: torch.Tensor):
        i = self._index.get(id(p))
        if i is not None:
            self._mark(i)

    # ------------------------------------------------------------------ API
    def forward(self, *args, **kw):
        return self.module(*args, **kw)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    def allreduce_grads(self):
        """Average gradients across ranks (call after the last micro-step's backward)."""
        if not is_dist() or not self._sync:
            return
        if self.grad_buffer is None:
            for p in self.module.parameters():
                if p.grad is not None:
                    all_reduce_mean_(p.grad)
            return
        if not self.overlap:
            for b in reversed(self.buckets()):
                all_reduce_mean_(b)
            return
        for b in range(self._next, len(self._buckets)):   # the tail, in order (some param got no gradient)
            self._launch(b, "flush")
        self._next = 0
        if self._stream is not None:
            cur = torch.cuda.current_stream(self.grad_buffer.device)
            ev0 = COMM.events(cur)          # the backward's last kernel is queued ahead of this point
            cur.wait_stream(self._stream)
            COMM.wait_end("all_reduce", ev0, cur)
        try:
            for work, view in self._works:
                t0 = time.perf_counter()
                work.wait()
                COMM.host_wait("all_reduce", time.perf_counter() - t0)
                view.div_(dist.get_world_size())
        finally:
            # the bucket state is reset even when a wait (or the poll below) raises: a caller that
            # handles the error and goes on must get all-reduces launched again next step
            self._works = []
            for bk in self._buckets:
                bk.launched = False
                bk.remaining = len(bk.params)
            self._ready = [False] * len(self._ready)
        if self.car is not None:
            self.car.poll()         # raises if a peer-memory reduction of the previous step timed out

    def reset_log(self):
        self.launch_log = []

    def close(self):
        """Release the peer-memory all-reduce (collective: every rank calls it)."""
        if self.car is not None:
            self.car.close()
            self.car = None


DDP = DistributedDataParallel
