"""hipGraph-captured decode steps (SURVEY.md K17 serving path; §7 "HIP graphs instead of a
tracing compiler").

One decode step of Qwen3-8B is ~450 kernel launches (36 layers × norm / fused QKV / qk-norm+RoPE
/ KV write / split-K attention + merge / o-proj+residual / norm / gate-up / SwiGLU / down+residual)
plus the LM head.  Launched eagerly from Python, the host-side dispatch cost (~10-20 µs per op)
exceeds the GPU time at small batch.  A :class:`DecodeGraphs` captures the whole step — embedding
through LM-head logits, including the in-place ``cache.pos += 1`` — once per batch bucket
(1, 2, 4, 8, 16, 32, 64, …) into a hipGraph and replays it: one host call per token.

Capture requirements the model code already meets: static shapes per bucket, the KV cache
pre-allocated (``KVCache`` rows ``[0, bucket)`` via :meth:`KVCache.head_rows`), per-row positions
kept on the device (no host sync), and the split-K decode-attention grid sized by the cache's
``max_len`` rather than the live lengths.  Inputs are copied into static buffers before replay.
"""
from __future__ import annotations

import torch

from ..models.common import KVCache
from ..ops.linear import head_logits


def _buckets(max_batch: int) -> list[int]:
    b, out = 1, []
    while b < max_batch:
        out.append(b)
        b *= 2
    out.append(max_batch)
    return out


class DecodeGraphs:
    """Capture ``lm.model`` + ``lm_head`` decode steps over ``cache`` for every batch bucket.

    ``step(tokens, n)`` runs rows ``[0, bucket(n))`` and returns logits ``[bucket, V]`` (a static
    buffer, valid until the next call)."""

    def __init__(self, lm, cache: KVCache, max_batch: int | None = None, buckets: list[int] | None = None,
                 tokens: torch.Tensor | None = None):
        self.lm, self.cache = lm, cache
        self.max_batch = max_batch or cache.batch
        self.buckets = buckets or _buckets(self.max_batch)
        dev = cache.k[0].device
        self.tokens = tokens if tokens is not None else torch.zeros(self.max_batch, dtype=torch.long, device=dev)
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.logits: dict[int, torch.Tensor] = {}
        self.pool = None
        self._capture_all()

    def _forward(self, n: int) -> torch.Tensor:
        h = self.lm.model(self.tokens[:n, None], None, self.cache.head_rows(n), None)
        return head_logits(h, self.lm.lm_head.weight)

    @torch.no_grad()
    def _capture_all(self):
        pos0 = self.cache.pos.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):          # warm up every bucket (allocator, lazy inits, kernels)
            for n in self.buckets:
                self._forward(n)
        torch.cuda.current_stream().wait_stream(s)
        for n in reversed(self.buckets):    # largest first: smaller graphs reuse its pool
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.pool):
                self.logits[n] = self._forward(n)
            if self.pool is None:
                self.pool = g.pool()
            self.graphs[n] = g
        self.cache.pos.copy_(pos0)          # warm-up and capture advanced the positions
        torch.cuda.synchronize()

    def bucket(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"batch {n} > max_batch {self.max_batch}")

    def step(self, tokens: torch.Tensor | None, n: int) -> torch.Tensor:
        """``tokens=None``: the caller already wrote the static ``self.tokens`` buffer."""
        b = self.bucket(n)
        if tokens is not None:
            self.tokens[:tokens.shape[0]].copy_(tokens)
        self.graphs[b].replay()
        return self.logits[b]
