"""Manual Python garbage collection for training loops.

The autograd graph of a step — above all under non-reentrant activation checkpointing, whose saved-tensor
hooks and recompute closures allocate thousands of Python objects per step — pushes CPython's generational
collector over its thresholds at arbitrary points of the step.  A generation-2 pass then walks every live
object of the process (the model, the optimizer, the data pipeline) while the GPU waits for the next launch:
a stall of several milliseconds at a random step.  The loop instead disables automatic collection and runs a
full collection itself every ``interval`` optimizer steps, at a step boundary (the role of Megatron-LM's
``--manual-gc``).  Reference cycles stay bounded: they are freed at the next interval.

    with ManualGC() as gcm:          # LIPA_GC_INTERVAL (default 100; 0 = leave Python's automatic GC on)
        for batch in loader:
            train_step(batch)
            gcm.step()
"""
from __future__ import annotations

import gc
import os


class ManualGC:
    def __init__(self, interval: int | None = None):
        self.interval = int(os.environ.get("LIPA_GC_INTERVAL", "100")) if interval is None else int(interval)
        self._was_enabled = None
        self._n = 0

    @property
    def active(self) -> bool:
        return self.interval > 0

    def __enter__(self):
        if self.active:
            self._was_enabled = gc.isenabled()
            gc.collect()
            gc.disable()
        return self

    def step(self):
        """Call once per optimizer step (at the step boundary)."""
        if not self.active:
            return
        self._n += 1
        if self._n % self.interval == 0:
            gc.collect()

    def __exit__(self, *exc):
        if self.active and self._was_enabled:
            gc.enable()
        return False
