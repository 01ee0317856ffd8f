"""Rank-aware logging.

Mirrors the reference's conventions: main-process-gated output
(``ddp_gpt_wikitext2.py:228-237``), a per-rank formatter plus an optional rank-0 file handler
``training.log`` (``temp/ddp_gpt_bpe_tokenizer_02.py:33-53``) and the ``LOG_LEVEL`` env var
(``GPTLike_wikitext2_fixed_pe.py:30-33``).
"""
from __future__ import annotations

import logging
import os
import sys


def _rank() -> int:
    return int(os.environ.get("RANK", "0"))


def get_logger(name: str = "lipa", log_file: str | None = None, all_ranks: bool = False) -> logging.Logger:
    log = logging.getLogger(name)
    if getattr(log, "_lipa_configured", False):
        return log
    level = getattr(logging, os.environ.get("LOG_LEVEL", "INFO").upper(), logging.INFO)
    r = _rank()
    log.setLevel(level if (all_ranks or r == 0) else logging.WARNING)
    fmt = logging.Formatter(f"%(asctime)s [rank{r}] %(levelname)s %(name)s: %(message)s")
    h = logging.StreamHandler(sys.stdout)
    h.setFormatter(fmt)
    log.addHandler(h)
    if log_file and r == 0:
        os.makedirs(os.path.dirname(os.path.abspath(log_file)), exist_ok=True)
        fh = logging.FileHandler(log_file)
        fh.setFormatter(fmt)
        log.addHandler(fh)
    log.propagate = False
    log._lipa_configured = True
    return log


def rank0_print(*a, **kw):
    if _rank() == 0:
        print(*a, **kw, flush=True)
