"""Host runtime under sanitizers: the CPU AdamW and the threaded token loader
built without bindings into ``tests/native/sanitize_host.cpp`` and run under ASan+UBSan and TSan."""
import concurrent.futures as cf
import shutil
import subprocess

import pytest

from llm_in_practise_amd.csrc.build import build_sanitizer_harness


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_runtime_clean_under_asan_ubsan_and_tsan():
    with cf.ThreadPoolExecutor(2) as ex:
        exes = list(ex.map(build_sanitizer_harness, ["address", "thread"]))
    for exe in exes:
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, f"{exe}\n{r.stdout}\n{r.stderr[-4000:]}"
        assert "all checks passed" in r.stdout
        assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
