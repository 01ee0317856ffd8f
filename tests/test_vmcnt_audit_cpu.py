"""The LDS-DMA kernels' counted vector-memory waits, checked structurally in their gfx950 ISA (CPU: hipcc -S).

Pins the fix of the round-5 dK/dV race (profiles/r5/zero3_dkv_race.txt): a register load issued beside LDS-DMAs
and guarded by a counted ``s_waitcnt vmcnt(N > 0)`` read stale data under contention.  The rule
(scripts/vmcnt_audit.py): while an LDS-DMA is outstanding, no counted wait may be what covers a register-
destination load.  Replaces the two-process GPU stress test that hoped to reproduce the race."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

pytestmark = pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not installed")


def test_audit_flags_the_race_pattern():
    """the checker itself: a counted wait covering a register load beside DMAs is flagged; the same wait
    covering only DMAs, and a full drain, are not"""
    from vmcnt_audit import audit
    bad = """k:
\tglobal_load_dwordx4 v[0:3], v[4:5], off
\tbuffer_load_dwordx4 v6, s[0:3], 0 offen lds
\tbuffer_load_dwordx4 v6, s[0:3], 0 offen lds
\ts_waitcnt vmcnt(2)
"""
    v, st = audit(bad)
    assert len(v) == 1 and st["counted_waits_beside_dma"] == 1
    ok = bad.replace("global_load_dwordx4 v[0:3], v[4:5], off", "buffer_load_dwordx4 v6, s[0:3], 0 offen lds")
    assert audit(ok)[0] == []
    assert audit(bad.replace("vmcnt(2)", "vmcnt(0)"))[0] == []
    assert audit(bad.replace("s_waitcnt vmcnt(2)", "s_waitcnt 0x3f72"))[0] != []   # raw gfx9 encoding, vmcnt 2


def test_lds_dma_kernels_have_no_counted_wait_on_register_loads():
    from vmcnt_audit import audit_sources
    res = audit_sources(cache_dir=os.path.join(ROOT, "build", "vmcnt_audit"))
    for src, (violations, stats) in res.items():
        assert stats["dma_ops"] > 0, src                    # the scan saw the kernels' DMAs
        assert stats["functions"] > 0
        assert not violations, f"{os.path.basename(src)}:\n" + "\n".join(violations[:10])
