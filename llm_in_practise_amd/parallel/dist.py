"""Process groups and collectives.

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` — which IS RCCL on ROCm,
running intra-node over xGMI (8×MI355X full mesh, 7 links/GPU) — or ``gloo`` on CPU.  Same
``env://`` contract as the reference (``ddp_gpt_wikitext2.py:170-182``): a missing
``WORLD_SIZE`` means single-process, and every helper degrades to a no-op.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..runtime.env import dist_env


def local_device_index(local_rank: int) -> int:
    """GPU of this rank: ``local_rank``, or ``local_rank % device_count`` under ``LIPA_SHARE_GPU=1``
    (a multi-rank rehearsal of the distributed path on a box with fewer GPUs than ranks; pair it with
    ``LIPA_DIST_BACKEND=gloo``, since RCCL refuses two ranks on one device)."""
    if os.environ.get("LIPA_SHARE_GPU", "0") == "1" and torch.cuda.is_available():
        return local_rank % max(1, torch.cuda.device_count())
    return local_rank


def init_distributed(backend: str | None = None, timeout_s: int = 1800) -> tuple[int, int, int]:
    """Initialise the default group from torchrun env vars.  Returns (rank, local_rank, world).
    ``LIPA_DIST_BACKEND`` overrides the backend (default: nccl = RCCL with GPUs, else gloo)."""
    env = dist_env()
    dev = local_device_index(env.local_rank)
    if env.world_size > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("LIPA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            torch.cuda.set_device(dev)
        kw = dict(backend=backend, init_method="env://", timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", dev)
        try:
            dist.init_process_group(**kw)
        except TypeError:
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(dev)
    return env.rank, env.local_rank, env.world_size


def comm_environment() -> dict:
    """What a multi-rank record needs to be reproduced: the collective library's version (RCCL on ROCm) and the
    NCCL_* / RCCL_* / TORCH_NCCL_* environment the run saw."""
    out: dict = {}
    try:
        if torch.cuda.is_available() and is_dist() and dist.get_backend() == "nccl":
            v = torch.cuda.nccl.version()
            out["rccl_version" if torch.version.hip else "nccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:   # pragma: no cover - the version query is informational
        out["rccl_version"] = f"unavailable ({type(e).__name__})"
    out["comm_env"] = {k: v for k, v in sorted(os.environ.items())
                       if k.startswith(("NCCL_", "RCCL_", "TORCH_NCCL_")) or k == "HSA_ENABLE_IPC_MODE_LEGACY"}
    return out


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def is_main() -> bool:
    return rank() == 0


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    if is_dist():
        if dist.get_backend(group) == "nccl" and hasattr(dist.ReduceOp, "AVG"):
            dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(t, group=group)
            t.div_(dist.get_world_size(group))
    return t


def all_reduce_max(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


class CommStats:
    """Per-step accounting of the data-parallel collectives, for the bench record (``COMM`` below).

    Per collective kind (``all_reduce`` / ``reduce_scatter`` / ``all_gather``):
      * ``calls`` and ``bytes`` issued;
      * ``busy_ms`` — time the collective itself ran, from CUDA events recorded on the stream that runs it
        (DDP's side stream; only where the framework owns that stream);
      * ``exposed_ms`` — time the compute stream stood waiting for collectives (CUDA events around the join
        on the GPU, host wall time of ``work.wait()`` on gloo).
    ``overlap_fraction`` = 1 − exposed / busy: the share of the communication hidden under the backward.
    Off unless ``enabled``; event pairs are resolved once, in :meth:`summary` (after a synchronise)."""

    KINDS = ("all_reduce", "reduce_scatter", "all_gather")

    def __init__(self):
        self.enabled = False
        self.reset()

    def reset(self):
        import collections
        self.calls = collections.Counter()
        self.bytes = collections.Counter()
        self._spans: list = []         # (kind, ev0, ev1): the collective's own run time
        self._waits: list = []         # (kind, ev0, ev1): compute stream stalled on it
        self._host_wait = collections.Counter()
        self.steps = 0

    def issue(self, kind: str, nbytes: int):
        if self.enabled:
            self.calls[kind] += 1
            self.bytes[kind] += int(nbytes)

    def events(self, stream=None):
        """(begin, end) recorder pair on ``stream`` (current stream if None), or None when off / on CPU."""
        if not (self.enabled and torch.cuda.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"):
            return None
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        return ev0

    def span_end(self, kind: str, ev0, stream=None):
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(stream)
            self._spans.append((kind, ev0, ev1))

    def wait_end(self, kind: str, ev0, stream=None):
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(stream)
            self._waits.append((kind, ev0, ev1))

    def host_wait(self, kind: str, seconds: float):
        if self.enabled:
            self._host_wait[kind] += seconds

    def step(self):
        if self.enabled:
            self.steps += 1

    def summary(self) -> dict:
        """Per-step means over the recorded steps (call after the device is synchronised)."""
        n = max(1, self.steps)
        busy = {k: 0.0 for k in self.KINDS}
        exposed = {k: 0.0 for k in self.KINDS}
        timed_busy = {k: False for k in self.KINDS}
        for kind, a, b in self._spans:
            busy[kind] += a.elapsed_time(b)
            timed_busy[kind] = True
        for kind, a, b in self._waits:
            exposed[kind] += a.elapsed_time(b)
        for kind, s in self._host_wait.items():
            exposed[kind] += 1000.0 * s
        out = {"steps": self.steps}
        tot_busy = tot_exp = 0.0
        for k in self.KINDS:
            if not self.calls[k]:
                continue
            rec = {"calls_per_step": round(self.calls[k] / n, 2), "mbytes_per_step": round(self.bytes[k] / n / 2 ** 20, 3),
                   "busy_ms_per_step": round(busy[k] / n, 3) if timed_busy[k] else None,
                   "exposed_ms_per_step": round(exposed[k] / n, 3)}
            out[k] = rec
            tot_exp += exposed[k] / n
            if timed_busy[k]:
                tot_busy += busy[k] / n
        out["exposed_ms_per_step"] = round(tot_exp, 3)
        out["overlap_fraction"] = (round(max(0.0, min(1.0, 1.0 - tot_exp / tot_busy)), 3) if tot_busy > 0 else None)
        return out


COMM = CommStats()
