"""Generation on CPU: KV-cache decoding == full recompute; sampler semantics (HF order)."""
import torch

from llm_in_practise_amd.infer.generate import GenerationConfig, generate, generate_simple
from llm_in_practise_amd.models.minigpt import MiniGPT
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.ops import reference as ref
from llm_in_practise_amd.ops.decode import (apply_repetition_penalty, decode_attention_reference,
                                            sample_reference)


def _naive_greedy(m, prompt, n):
    ids = prompt.clone()
    for _ in range(n):
        logits = m(ids[None]).logits[0, -1]
        ids = torch.cat([ids, logits.argmax()[None]])
    return ids


def test_kv_cache_greedy_matches_recompute_with_ragged_batch():
    torch.manual_seed(0)
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, seed=0).eval()
    p0 = torch.randint(0, 512, (7,))
    p1 = torch.randint(0, 512, (4,))
    ids = torch.zeros(2, 7, dtype=torch.long)
    am = torch.zeros(2, 7, dtype=torch.long)
    ids[0], am[0] = p0, 1
    ids[1, :4], am[1, :4] = p1, 1
    out = generate(m, ids, am, max_new_tokens=6, do_sample=False, pad_token_id=0)
    assert torch.equal(out[0, :13], _naive_greedy(m, p0, 6))
    assert torch.equal(out[1, :10], _naive_greedy(m, p1, 6))


def test_generate_stops_at_eos_and_pads():
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, seed=1).eval()
    p = torch.randint(0, 512, (1, 5))
    first = generate(m, p, max_new_tokens=1)[0, 5].item()
    out = generate(m, p, max_new_tokens=10, eos_token_id=first, pad_token_id=3, sync_every=1)
    assert out.shape[1] == 6 and out[0, 5].item() == first


def test_decode_attention_reference_matches_full_attention():
    torch.manual_seed(0)
    B, Smax, hq, hkv, d = 2, 20, 8, 2, 16
    kc, vc = torch.randn(B, Smax, hkv * d), torch.randn(B, Smax, hkv * d)
    q = torch.randn(B, hq * d)
    lens = torch.tensor([20, 11])
    o = decode_attention_reference(q, kc, vc, lens, hq, hkv, d)
    for b in range(B):
        L = int(lens[b])
        r = ref.attention(q[b].view(1, 1, hq, d), kc[b, :L].view(1, L, hkv, d), vc[b, :L].view(1, L, hkv, d),
                          causal=False)
        assert torch.allclose(o[b], r.reshape(-1), atol=1e-5)


def test_sampler_semantics():
    torch.manual_seed(0)
    logits = torch.randn(4, 50)
    g = torch.argmax(logits, -1)
    assert torch.equal(sample_reference(logits, temperature=0), g)
    assert torch.equal(sample_reference(logits, temperature=1.0, top_k=1), g)
    assert torch.equal(sample_reference(logits, temperature=0.7, top_p=1e-6), g)
    # penalty applied once per distinct token, sign-aware
    x = torch.tensor([[2.0, -2.0, 1.0]])
    h = torch.tensor([[0, 0, 1, -1]])
    y = apply_repetition_penalty(x, h, 2.0)
    assert torch.allclose(y, torch.tensor([[1.0, -4.0, 1.0]]))
    # top-p keeps the smallest top set with mass >= p
    lg = torch.log(torch.tensor([[0.5, 0.3, 0.15, 0.05]]))
    draws = torch.stack([sample_reference(lg, temperature=1.0, top_p=0.7) for _ in range(300)])
    assert set(draws.unique().tolist()) <= {0, 1}


def test_generate_simple_minigpt_greedy_window():
    torch.manual_seed(0)
    m = MiniGPT(30).eval()
    idx = torch.randint(0, 30, (1, 20))
    out = generate_simple(m, idx, 5, block_size=16)
    assert out.shape == (1, 25)
    nxt = m(out[:, 20 - 16 + 0:20])[:, -1].argmax(-1)
    assert nxt.item() == out[0, 20].item()


def test_rope_table_cache_matches_explicit_positions():
    """Qwen3Model caches the cos / sin tables of positions 0 .. S-1 per (B, S): the default-position forward
    equals the forward with explicit position ids, call after call and across shapes"""
    import torch
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    lm = Qwen3ForCausalLM.from_config(qwen3_config("qwen2-tiny"), dtype=torch.float32, seed=0).eval()
    with torch.no_grad():
        for B, S in ((2, 7), (1, 16), (2, 7)):
            ids = torch.randint(0, 512, (B, S))
            pos = torch.arange(S).expand(B, S)
            a = lm.model(ids)
            b = lm.model(ids, pos)
            assert torch.equal(a, b)
    assert len(lm.model._rope_cache) == 2
