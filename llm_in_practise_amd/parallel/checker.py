"""Collective-sequence checker (SURVEY.md §5.2 MI355X plan).

The reference has latent collective-order bugs: a rank-0-only extra ``dist.barrier()``
(``temp/ddp_gpt_bpe_tokenizer.py:369-387``) and a rank-0-only ``save_checkpoint``
(``DeepSpeed/temp/DeepSpeed-GPTLike-bpe-wikitext2.py:321-323``).  Under RCCL such mismatches
hang or silently pair unrelated collectives.  In debug mode this checker wraps the
``torch.distributed`` collectives; before a collective is issued, every ``every``-th call
exchanges a digest of ``(seq, op, shape, dtype)`` with all ranks (one tiny all-gather on
the *same* process group, issued through the original function) and raises
:class:`CollectiveMismatch` naming the diverging ranks instead of hanging.

    with CollectiveChecker(every=1):
        train()

Also enabled by ``LIPA_CHECK_COLLECTIVES=<every>`` through :func:`maybe_enable`.
"""
from __future__ import annotations

import hashlib
import os

import torch
import torch.distributed as dist

_WRAPPED = ("all_reduce", "broadcast", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor",
            "reduce_scatter", "reduce", "barrier", "all_to_all_single", "gather", "scatter")


class CollectiveMismatch(RuntimeError):
    pass


def _describe(op, args, kw):
    parts = [op]
    for a in list(args) + list(kw.values()):
        if isinstance(a, torch.Tensor):
            parts.append(f"{tuple(a.shape)}:{a.dtype}")
        elif isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
            parts.append(f"[{len(a)}x{tuple(a[0].shape)}:{a[0].dtype}]")
    return "|".join(parts)


class CollectiveChecker:
    def __init__(self, every: int = 1):
        self.every = max(1, every)
        self.seq = 0
        self.log: list[str] = []
        self._orig = {}

    def _digest_check(self, desc, group):
        h = int.from_bytes(hashlib.sha1(f"{self.seq}:{desc}".encode()).digest()[:7], "little")
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if dist.get_backend(group) == "nccl" else torch.device("cpu")
        mine = torch.tensor([h], dtype=torch.int64, device=dev)
        allh = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
        self._orig["all_gather"](allh, mine, group=group)
        vals = [int(t.item()) for t in allh]
        if len(set(vals)) != 1:
            bad = [i for i, v in enumerate(vals) if v != vals[dist.get_rank(group) if group else 0]]
            raise CollectiveMismatch(f"collective #{self.seq} '{desc}' on rank {dist.get_rank()} diverges from "
                                     f"ranks {bad}; recent: {self.log[-5:]}")

    def _wrap(self, name):
        orig = self._orig[name]

        def fn(*args, **kw):
            desc = _describe(name, args, kw)
            self.seq += 1
            self.log.append(desc)
            if self.seq % self.every == 0:
                self._digest_check(desc, kw.get("group"))
            return orig(*args, **kw)
        return fn

    def __enter__(self):
        for n in _WRAPPED:
            if hasattr(dist, n):
                self._orig[n] = getattr(dist, n)
        for n in list(self._orig):
            setattr(dist, n, self._wrap(n))
        return self

    def __exit__(self, *exc):
        for n, f in self._orig.items():
            setattr(dist, n, f)
        return False


def maybe_enable():
    every = os.environ.get("LIPA_CHECK_COLLECTIVES")
    if every and dist.is_available() and dist.is_initialized():
        c = CollectiveChecker(int(every))
        c.__enter__()
        return c
    return None
