"""Numerical parity with the HF ``transformers`` implementations the reference scripts load
(``AutoModelForCausalLM.from_pretrained`` on Qwen3-8B/14B, DeepSeek-R1-0528-Qwen3-8B and the
Qwen2-architecture DeepSeek-R1-Distill-Qwen-1.5B; SURVEY.md §2.1 Tracks E/G).

Tiny random-init HF models are built locally (no download), their state dict is loaded into
our model through the same ``load_hf_state_dict`` / safetensors path a real checkpoint uses,
and logits / loss are compared on the CPU reference path (fp32).
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from llm_in_practise_amd.models.qwen3 import Qwen3Config, Qwen3ForCausalLM  # noqa: E402


def _hf_tiny(kind: str):
    common = dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                  rms_norm_eps=1e-6, tie_word_embeddings=False)
    if kind == "qwen3":
        cfg = transformers.Qwen3Config(head_dim=32, **common)
        cls = transformers.Qwen3ForCausalLM
    else:
        cfg = transformers.Qwen2Config(**common)
        cls = transformers.Qwen2ForCausalLM
    cfg._attn_implementation = "eager"
    torch.manual_seed(0)
    m = cls(cfg).float().eval()
    with torch.no_grad():   # HF zero-inits some params; randomise everything so parity is non-trivial
        for n, p in m.named_parameters():
            if "norm" in n:
                p.copy_(1 + 0.1 * torch.randn_like(p))
            else:
                p.normal_(0, 0.05)
    return m


@pytest.mark.parametrize("kind", ["qwen3", "qwen2"])
def test_logits_and_loss_match_transformers(kind):
    hf = _hf_tiny(kind)
    cfg = Qwen3Config.from_dict(hf.config.to_dict())
    assert cfg.qk_norm == (kind == "qwen3") and cfg.attention_bias == (kind == "qwen2")
    ours = Qwen3ForCausalLM(cfg).float().eval()
    missing = ours.load_hf_state_dict(hf.state_dict(), strict=True)
    assert not missing
    ids = torch.randint(0, 512, (2, 24))
    with torch.no_grad():
        ref = hf(ids, labels=ids)
        out = ours(ids, labels=ids, return_logits=True)
    err = (out.logits - ref.logits).abs().max() / ref.logits.abs().max()
    assert err < 1e-4, f"{kind}: logits rel err {err:.2e}"
    assert abs(out.loss.item() - ref.loss.item()) < 1e-4 * abs(ref.loss.item())


@pytest.mark.parametrize("kind", ["qwen3", "qwen2"])
def test_save_pretrained_roundtrip_loads_in_transformers(kind, tmp_path):
    """Our ``save_pretrained`` writes an HF-layout dir that transformers loads back unchanged."""
    hf = _hf_tiny(kind)
    cfg = Qwen3Config.from_dict(hf.config.to_dict())
    ours = Qwen3ForCausalLM(cfg).float().eval()
    ours.load_hf_state_dict(hf.state_dict(), strict=True)
    ours.save_pretrained(str(tmp_path))
    back = Qwen3ForCausalLM.from_pretrained(str(tmp_path), dtype=torch.float32).eval()
    ids = torch.randint(0, 512, (1, 16))
    with torch.no_grad():
        a = ours(ids).logits
        b = back(ids).logits
    assert torch.allclose(a, b)
    cls = transformers.Qwen3ForCausalLM if kind == "qwen3" else transformers.Qwen2ForCausalLM
    hf2 = cls.from_pretrained(str(tmp_path), torch_dtype=torch.float32).eval()
    with torch.no_grad():
        c = hf2(ids).logits
    assert (a - c).abs().max() / c.abs().max() < 1e-4
