"""Progress watchdog for multi-rank runs (SURVEY.md §5.3 failure detection).

A collective that never completes (a peer died, OOM'd, or took a different code path) blocks the calling
thread inside RCCL / gloo until the process group's timeout — 30 minutes by default, far past any driver or
scheduler budget, and with nothing on stderr to say where it stopped.  ``Watchdog`` is a daemon thread with
a deadline that the main thread pushes forward (``beat``) while it makes progress.  When the deadline
passes it writes a diagnostic (rank, phase, seconds without progress, every thread's Python stack), runs an
optional ``on_expire`` callback (``bench.py`` prints its already-measured headline record there) and ends
the process with ``os._exit`` — no Python teardown that could itself block on the stuck collective.

The process group's own timeout stays configured as the last resort (``parallel/dist.py``).
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time


class Watchdog:
    def __init__(self, rank: int = 0, poll_s: float = 0.25):
        self.rank = rank
        self.poll_s = poll_s
        self._lock = threading.Lock()
        self._deadline: float | None = None
        self._budget = 0.0
        self._label = ""
        self._on_expire = None
        self._exit_code = 3
        self._thread: threading.Thread | None = None
        self.fired = False

    def arm(self, seconds: float, label: str, on_expire=None, exit_code: int = 3):
        """Start (or restart) the countdown: ``seconds`` without a ``beat`` ends the process."""
        with self._lock:
            self._budget = float(seconds)
            self._deadline = time.monotonic() + self._budget
            self._label = label
            self._on_expire = on_expire
            self._exit_code = exit_code
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name="lipa-watchdog", daemon=True)
                self._thread.start()

    def beat(self):
        with self._lock:
            if self._deadline is not None:
                self._deadline = time.monotonic() + self._budget

    def disarm(self):
        with self._lock:
            self._deadline = None
            self._on_expire = None

    @property
    def armed(self) -> bool:
        return self._deadline is not None

    def _run(self):
        while True:
            time.sleep(self.poll_s)
            with self._lock:
                dl = self._deadline
                if dl is None or time.monotonic() < dl:
                    continue
                label, budget, cb, code = self._label, self._budget, self._on_expire, self._exit_code
                self._deadline = None
                self.fired = True
            self._fire(label, budget, cb, code)

    def _fire(self, label, budget, cb, code):
        try:
            print(f"[watchdog] rank {self.rank}: no progress in '{label}' for {budget:.0f} s "
                  f"(collective stall, dead peer or hang); stacks follow, exiting with {code}",
                  file=sys.stderr, flush=True)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:   # pragma: no cover - diagnostics must never block the exit
            pass
        if cb is not None:
            try:
                cb()
            except Exception as e:   # pragma: no cover
                print(f"[watchdog] on_expire failed: {e!r}", file=sys.stderr, flush=True)
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        finally:
            os._exit(code)
