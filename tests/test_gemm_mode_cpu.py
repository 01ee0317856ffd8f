"""One GEMM form: every frozen-base GEMM at training size is the hand-written gemm4w — no library GEMM mode,
no LIPA_GEMM / LIPA_LT dispatch (ops/gemm.py); torch.matmul only for shapes gemm4w does not take, and
GEMM_STATS says which form every launch took (the bench record's provenance)."""
import torch

import llm_in_practise_amd.ops.gemm as G
import llm_in_practise_amd.ops.linear as L


def test_no_library_gemm_modes():
    """and no losing LoRA variants kept behind knobs: one kernel form per adapter layout (ops/linear.py)"""
    for name in ("_GEMM_MODE", "_LT", "_g4w_on", "_APPLY", "_LORA_EPI", "_dx_split", "_KEEP_BITS", "_PAIR_BWD",
                 "_DX_C"):
        assert not hasattr(L, name) and not hasattr(G, name), name
    for mod in (L, G):
        src = open(mod.__file__).read()
        for knob in ("LIPA_GEMM", "LIPA_LT", "LIPA_LORA_APPLY", "LIPA_LORA_EPI", "LIPA_LORA_PAIR", "LIPA_LORA_MULTI",
                     "lt_linear", "lt_dx", "lora_acc2"):
            assert knob not in src, knob


def test_no_runtime_switches_in_attention_kernels():
    """one attention kernel per (head-dim class, pass): no environment-read A/B switches in the shipped .so"""
    import os
    src = open(os.path.join(os.path.dirname(L.__file__), "..", "csrc", "kernels", "attention.hip")).read()
    assert "getenv" not in src


def test_gemm_stats_count_forms():
    L.GEMM_STATS.clear()
    x = torch.randn(8, 64)
    w = torch.randn(32, 64)
    y = L._base_gemm(x, w)                       # CPU: gemm4w does not take it -> counted as the fallback
    assert torch.allclose(y, x @ w.t())
    dx = G._dense_dx(torch.randn(8, 32), w)
    assert dx.shape == (8, 64)
    assert L.GEMM_STATS["library"] == 2 and L.GEMM_STATS["gemm4w"] == 0
    L.GEMM_STATS.clear()
