"""The kept opt-in variants stay numerically equivalent to the default path, so their A/B records
(profiles/) compare like with like: the unfused SwiGLU MLP (LIPA_FUSED_MLP=0) and
hipBLASLt in place of every hand-written gemm4w GEMM (LIPA_GEMM=lt) and gemm4w for every one (LIPA_GEMM=native;
the default, hybrid, keeps it where the LoRA terms ride in the GEMM), and the memory-lean NF4 mode that
feeds every NF4 GEMM the 4-bit codes (LIPA_NF4_GEMM=w4).  Each runs the bench step on a small Qwen3 in a
subprocess (the switches are read once per process).  The measured-slower scheduling variants of
round 2 (side-stream LoRA projection, two-stream attention backward, background NF4 expansion,
deferred attention max, multi-adapter dx-as-C) were deleted; their records stay in profiles/."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _losses(extra_env):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", **extra_env)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "qwen3-small", "--steps", "3",
                          "--warmup", "1", "--faithful-steps", "0"], env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    return [float(x) for x in re.findall(r"loss=([0-9.]+)", out.stderr)]


@pytest.fixture(scope="module")
def base_losses():
    got = _losses({})
    assert len(got) == 2
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"LIPA_FUSED_MLP": "0"}, {"LIPA_GEMM": "lt"}, {"LIPA_GEMM": "native"},
                                 {"LIPA_NF4_GEMM": "w4"}],
                         ids=lambda e: ",".join(e))
def test_opt_in_schedule_matches_default(base_losses, env):
    got = _losses(env)
    assert len(got) == 2 and all(abs(a - b) <= 2e-3 * abs(b) for a, b in zip(got, base_losses)), (env, got,
                                                                                                   base_losses)
