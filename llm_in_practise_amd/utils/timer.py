"""Step timer with a DeepSpeed ``wall_clock_breakdown``-style phase split.

On GPU each phase is bracketed by HIP events on the current stream, so timing does not add
host synchronisation inside the step; ``summary()`` synchronises once and converts.  On CPU
it falls back to ``time.perf_counter``.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch


class StepTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.gpu = torch.cuda.is_available()
        self._events = defaultdict(list)
        self._cpu = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.gpu:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._events[name].append((a, b))
        else:
            t = time.perf_counter()
            yield
            self._cpu[name] += (time.perf_counter() - t) * 1e3

    def summary(self, reset: bool = True) -> dict[str, float]:
        """Milliseconds per phase accumulated since the last reset."""
        out = dict(self._cpu)
        if self._events:
            torch.cuda.synchronize()
            for k, evs in self._events.items():
                out[k] = out.get(k, 0.0) + sum(a.elapsed_time(b) for a, b in evs)
        if reset:
            self._events.clear()
            self._cpu.clear()
        return out
