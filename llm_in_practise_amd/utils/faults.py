"""Fault injection for resume / failure-detection tests (SURVEY.md §5.3 MI355X plan).

``FAULT_INJECT=rank:step:kind[,rank:step:kind...]`` where kind is
  * ``raise`` — raise :class:`InjectedFault` at that optimizer step (tests the trainer's
    ``_interrupted`` save and ``resume_from_checkpoint``),
  * ``nan``   — poison the loss with NaN (tests non-finite handling / fp16 overflow skip),
  * ``hang``  — sleep ``FAULT_HANG_S`` seconds (default 3600) so collective timeouts fire,
  * ``exit``  — ``os._exit(17)`` (tests torchrun ``--max-restarts`` elastic restarts).
``rank`` may be ``*`` for all ranks.
"""
from __future__ import annotations

import os
import time


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, spec: str | None = None, rank: int | None = None):
        spec = spec if spec is not None else os.environ.get("FAULT_INJECT", "")
        self.rank = rank if rank is not None else int(os.environ.get("RANK", "0"))
        self.rules = []
        for item in filter(None, (s.strip() for s in spec.split(","))):
            r, s, kind = item.split(":")
            self.rules.append((None if r == "*" else int(r), int(s), kind))
        self.fired = set()

    def __bool__(self):
        return bool(self.rules)

    def check(self, step: int) -> str | None:
        """Return ``"nan"`` when the loss should be poisoned; raise/hang/exit otherwise."""
        for i, (r, s, kind) in enumerate(self.rules):
            if i in self.fired or s != step or (r is not None and r != self.rank):
                continue
            self.fired.add(i)
            if kind == "raise":
                raise InjectedFault(f"injected fault at rank {self.rank} step {step}")
            if kind == "hang":
                time.sleep(float(os.environ.get("FAULT_HANG_S", "3600")))
            elif kind == "exit":
                os._exit(17)
            elif kind == "nan":
                return "nan"
        return None
