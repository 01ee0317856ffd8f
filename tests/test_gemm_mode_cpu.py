"""One GEMM form: every frozen-base GEMM at training size is the hand-written gemm4w — no library GEMM mode,
no LIPA_GEMM / LIPA_LT dispatch (ops/linear.py); torch.matmul only for shapes gemm4w does not take, and
GEMM_STATS says which form every launch took (the bench record's provenance)."""
import torch

import llm_in_practise_amd.ops.linear as L


def test_no_library_gemm_modes():
    for name in ("_GEMM_MODE", "_LT", "_g4w_on", "_APPLY", "_LORA_EPI", "_dx_split"):
        assert not hasattr(L, name), name
    src = open(L.__file__).read()
    for knob in ("LIPA_GEMM", "LIPA_LT", "LIPA_LORA_APPLY", "LIPA_LORA_EPI", "LIPA_LORA_PAIR", "LIPA_LORA_MULTI",
                 "lt_linear", "lt_dx"):
        assert knob not in src, knob


def test_gemm_stats_count_forms():
    L.GEMM_STATS.clear()
    x = torch.randn(8, 64)
    w = torch.randn(32, 64)
    y = L._base_gemm(x, w)                       # CPU: gemm4w does not take it -> counted as the fallback
    assert torch.allclose(y, x @ w.t())
    dx = L._dense_dx(torch.randn(8, 32), w)
    assert dx.shape == (8, 64)
    assert L.GEMM_STATS["library"] == 2 and L.GEMM_STATS["gemm4w"] == 0
    L.GEMM_STATS.clear()
