"""The per-role GEMM policy (ops/linear.py ``_g4w_on``, LIPA_GEMM): hybrid (default) keeps the hand-written
gemm4w where work rides inside it — the LoRA prologues (lora=True) and checkpointed layers — and sends the
plain bf16 GEMMs to hipBLASLt; native / lt are all-gemm4w / all-library."""
import llm_in_practise_amd.ops.linear as L


def test_gemm_mode_policy(monkeypatch):
    monkeypatch.setattr(L, "_GEMM_MODE", "hybrid")
    assert L._g4w_on(lora=True) and not L._g4w_on()
    monkeypatch.setattr(L, "_IN_CKPT", [1])
    assert L._g4w_on() and L._g4w_on(lora=True)
    monkeypatch.setattr(L, "_IN_CKPT", [0])
    monkeypatch.setattr(L, "_GEMM_MODE", "native")
    assert L._g4w_on() and L._g4w_on(lora=True)
    monkeypatch.setattr(L, "_GEMM_MODE", "lt")
    assert not L._g4w_on() and not L._g4w_on(lora=True)


def test_default_mode_is_hybrid():
    import os
    if "LIPA_GEMM" not in os.environ:
        assert L._GEMM_MODE == "hybrid"
