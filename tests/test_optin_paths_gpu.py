"""The kept variants stay numerically equivalent to the default path, so their A/B records (profiles/) compare
like with like: the unfused SwiGLU MLP (separate projections + activation kernels: models/qwen3.py
``_FUSED_MLP``), and the two NF4 forms — the memory-lean mode that feeds every NF4 GEMM the 4-bit codes
(``--nf4-gemm w4``) and one bf16 expansion per weight (``--nf4-gemm expand``).  Each runs the bench step on a
small Qwen3 in a subprocess; the JSON's config records the NF4 form that ran."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _losses(args=(), code=None, want_nf4=None):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("LIPA_NF4_GEMM", None)
    cmd = [sys.executable, "-c", code, *args] if code else [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    out = subprocess.run(cmd + ["--model", "qwen3-small", "--steps", "3", "--warmup", "1", "--faithful-steps", "0",
                                "--selective-steps", "0"], env=env, capture_output=True, text=True, timeout=110,
                         cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    if want_nf4 is not None:
        rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
        assert rec["config"]["nf4_gemm"] == want_nf4, rec["config"]
    return [float(x) for x in re.findall(r"loss=([0-9.]+)", out.stderr)]


# bench.py with the fused MLP switched off (the switch is a module constant, set before the model is built)
_UNFUSED = ("import sys, runpy; sys.argv = ['bench.py'] + sys.argv[1:]; "
            "import llm_in_practise_amd.models.qwen3 as q; q._FUSED_MLP = False; "
            "runpy.run_path('bench.py', run_name='__main__')")


@pytest.fixture(scope="module")
def base_losses():
    got = _losses()
    assert len(got) == 2
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["unfused-mlp", "nf4-w4", "nf4-expand"])
def test_opt_in_schedule_matches_default(base_losses, variant):
    if variant == "unfused-mlp":
        got = _losses(code=_UNFUSED)
    else:
        mode = variant.split("-")[1]
        got = _losses(["--nf4-gemm", mode], want_nf4=mode)
    assert len(got) == 2 and all(abs(a - b) <= 2e-3 * abs(b) for a, b in zip(got, base_losses)), (variant, got,
                                                                                                   base_losses)
