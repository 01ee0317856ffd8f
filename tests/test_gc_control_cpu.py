"""Manual GC for training loops (utils/gc_control.py): automatic collection off inside, a full pass every
`interval` steps, the previous state restored on exit; interval 0 leaves Python's GC alone."""
import gc

from llm_in_practise_amd.utils.gc_control import ManualGC


def test_manual_gc_disables_and_restores():
    assert gc.isenabled()
    calls = []
    orig = gc.collect
    try:
        gc.collect = lambda *a: calls.append(a) or 0
        with ManualGC(3) as g:
            assert not gc.isenabled()
            for _ in range(7):
                g.step()
        assert len(calls) == 1 + 2          # on entry, then at steps 3 and 6
    finally:
        gc.collect = orig
    assert gc.isenabled()


def test_manual_gc_interval_zero_is_a_no_op():
    with ManualGC(0) as g:
        assert gc.isenabled()
        g.step()
    assert gc.isenabled()
