"""Data parallel: ``DDP(model, device_ids=[local_rank])`` semantics.

MI355X design: gradients live in ONE flat fp32 buffer (owned by the fused optimizer, see
``optim/adamw.py``), so the data-parallel reduction is bucketed over that buffer and never
packs/unpacks.  Buckets are sized for xGMI rings (default 64 MiB, far larger than torch's
25 MiB: intra-node RCCL rings are per-link bandwidth-bound, so fewer, larger collectives
win); LoRA-sized buffers (15-60 MB) are a single collective.  Buckets are issued on a
side stream in reverse layer order after the boundary micro-step's backward;
``no_sync()`` skips the reduction on non-boundary gradient-accumulation micro-steps.

On start the module's parameters and buffers are broadcast from rank 0
(``sync_module_states``).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import all_reduce_mean_, is_dist


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, grad_buffer: torch.Tensor | None = None, bucket_mb: float = 64.0,
                 broadcast_buffers: bool = True, device_ids=None, find_unused_parameters: bool = False,
                 overlap: bool = True, **_):
        super().__init__()
        self.module = module
        self.grad_buffer = grad_buffer
        self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
        self._sync = True
        self._pending = []
        self.overlap = overlap and grad_buffer is not None and torch.cuda.is_available()
        if is_dist():
            with torch.no_grad():
                for t in list(module.parameters()) + (list(module.buffers()) if broadcast_buffers else []):
                    dist.broadcast(t.data, src=0)
        self._stream = torch.cuda.Stream() if self.overlap else None

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

    def buckets(self) -> list[torch.Tensor]:
        g = self.grad_buffer
        return [g[s:s + self.bucket_elems] for s in range(0, g.numel(), self.bucket_elems)]

    def allreduce_grads(self):
        """Average gradients across ranks (call after the last micro-step's backward)."""
        if not is_dist() or not self._sync:
            return
        if self.grad_buffer is None:
            for p in self.module.parameters():
                if p.grad is not None:
                    all_reduce_mean_(p.grad)
            return
        if self.overlap:
            cur = torch.cuda.current_stream()
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                for b in reversed(self.buckets()):
                    all_reduce_mean_(b)
            cur.wait_stream(self._stream)
        else:
            for b in self.buckets():
                all_reduce_mean_(b)


DDP = DistributedDataParallel
