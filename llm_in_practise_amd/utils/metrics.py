"""Structured per-step metrics (SURVEY.md §5.5 MI355X plan): one JSON object per line.

Fields written by the trainer: step, epoch, loss, lr, grad_norm, tokens (padded and
non-pad), tokens_per_s, step_ms, phase times (fwd_bwd/comm/optim), peak HBM GiB.
"""
from __future__ import annotations

import json
import os
import time


class MetricsWriter:
    def __init__(self, path: str | None, rank: int = 0):
        self.path = path if rank == 0 else None
        self._f = None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a", buffering=1)

    def write(self, **rec):
        if self._f is None:
            return
        rec.setdefault("time", time.time())
        self._f.write(json.dumps(rec, default=float) + "\n")

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]
