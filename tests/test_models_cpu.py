"""Teaching-model zoo vs torch.nn oracles (CPU): reference state dicts load and give the same outputs."""
import math

import pytest
import torch
import torch.nn as nn

from llm_in_practise_amd.models import layers as L
from llm_in_practise_amd.models.deepseeklike import DeepSeekLike
from llm_in_practise_amd.models.gptlike import GPTLike, SimpleTransformer
from llm_in_practise_amd.models.minigpt import MiniGPT, MiniGPT2, MiniGPT2Config


class RefMiniGPT(nn.Module):
    """Oracle with the reference's structure (llm-demo/minigpt/model.py) built from torch.nn."""

    def __init__(self, vocab, d=64, h=2, n=2):
        super().__init__()
        self.token_embed = nn.Embedding(vocab, d)
        self.pos_embed = nn.Embedding(16, d)
        self.layers = nn.ModuleList([nn.TransformerDecoderLayer(d_model=d, nhead=h, dropout=0.1) for _ in range(n)])
        self.register_buffer("dummy_memory", torch.zeros(1, 1, d))
        self.fc = nn.Linear(d, vocab)

    def forward(self, x):
        pos = torch.arange(0, x.size(1))
        x = self.token_embed(x) + self.pos_embed(pos)
        mem = self.dummy_memory.expand(x.size(0), x.size(1), -1)
        for layer in self.layers:
            x = layer(x, mem)
        return self.fc(x)


def test_minigpt_reproduces_reference_exactly():
    torch.manual_seed(0)
    ref = RefMiniGPT(40).eval()
    ours = MiniGPT(40).eval()
    missing = ours.load_state_dict(ref.state_dict(), strict=True)
    x = torch.randint(0, 40, (4, 16))
    assert torch.allclose(ours(x), ref(x), atol=1e-5)


def test_minigpt_causal_variant_is_causal():
    torch.manual_seed(0)
    m = MiniGPT(40, reference_layout=False, causal=True).eval()
    x = torch.randint(0, 40, (2, 16))
    y1 = m(x)
    x2 = x.clone()
    x2[:, 10:] = (x2[:, 10:] + 1) % 40
    y2 = m(x2)
    assert torch.allclose(y1[:, :10], y2[:, :10], atol=1e-5)


def test_minigpt2_matches_nn_encoder():
    torch.manual_seed(0)
    cfg = MiniGPT2Config(seq_len=32, vocab_size=50)
    ours = MiniGPT2(cfg).eval()
    enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(128, 4, 512, 0.1, activation="gelu", batch_first=True), 4)
    enc.load_state_dict(ours.transformer.state_dict())
    enc.eval()
    x = torch.randint(0, 50, (2, 32))
    h = ours.embed(x) + ours.pos_embed
    ref = ours.head(ours.ln(enc(h)))
    assert torch.allclose(ours(x), ref, atol=1e-5)


class RefGPTLike(nn.Module):
    def __init__(self, V, block, n, h, d):
        super().__init__()
        self.tok_emb = nn.Embedding(V, d)
        self.blocks = nn.ModuleList()
        for _ in range(n):
            blk = nn.Module()
            blk.ln1, blk.ln2 = nn.LayerNorm(d), nn.LayerNorm(d)
            blk.attn = nn.Module()
            blk.attn.mha = nn.MultiheadAttention(d, h, batch_first=True)
            blk.mlp = nn.Module()
            blk.mlp.net = nn.Sequential(nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d), nn.Dropout(0.1))
            self.blocks.append(blk)
        self.ln_f = nn.LayerNorm(d)
        self.head = nn.Linear(d, V, bias=False)
        self.head.weight = self.tok_emb.weight

    def forward(self, idx, pe):
        x = self.tok_emb(idx) + pe[:, :idx.shape[1]]
        Lq = idx.shape[1]
        mask = torch.triu(torch.ones(Lq, Lq), 1).bool()
        for b in self.blocks:
            h = b.ln1(x)
            x = x + b.attn.mha(h, h, h, attn_mask=mask)[0]
            x = x + b.mlp.net(b.ln2(x))
        return self.head(self.ln_f(x))


def test_gptlike_matches_reference_structure():
    torch.manual_seed(0)
    ours = GPTLike(100, 32, 2, 4, 64).eval()
    ref = RefGPTLike(100, 32, 2, 4, 64).eval()
    sd = ours.state_dict()
    ref.load_state_dict({k: v for k, v in sd.items() if k != "pos_emb"}, strict=True)
    x = torch.randint(0, 100, (3, 20))
    assert torch.allclose(ours(x), ref(x, ours.pos_emb), atol=1e-5)
    _, loss = ours(x, torch.roll(x, -1, 1))
    ref_loss = nn.functional.cross_entropy(ref(x, ours.pos_emb).reshape(-1, 100), torch.roll(x, -1, 1).reshape(-1))
    assert abs(loss.item() - ref_loss.item()) < 1e-4


def test_gptlike_param_count_matches_survey():
    m = GPTLike.from_preset("gptlike-bert")
    assert abs(m.num_params() - 65.97e6) / 65.97e6 < 0.005       # SURVEY C: ≈65.97 M


def test_gptlike_learned_pe_and_resize():
    m = GPTLike.from_preset("gpt-byte", n_layer=1)
    assert isinstance(m.pos_emb, nn.Embedding)
    m.resize_token_embeddings(300)
    assert m.head.weight is m.tok_emb.weight and m(torch.randint(0, 300, (1, 8))).shape == (1, 8, 300)


def test_simple_transformer_shapes():
    m = SimpleTransformer(50, d_model=32, nhead=4, num_layers=2, max_len=16)
    assert m(torch.randint(0, 50, (2, 16))).shape == (2, 16, 50)


def test_deepseeklike_forward_backward_and_moe_dispatch_equivalence():
    torch.manual_seed(0)
    m = DeepSeekLike(vocab_size=64, block_size=32, n_layer=2, n_head=4, d_model=64, dropout=0.0)
    x = torch.randint(0, 64, (2, 16))
    _, loss = m(x, torch.roll(x, -1, 1))
    loss.backward()
    assert math.isfinite(loss.item()) and m.tok_emb.weight.grad is not None
    moe = m.blocks[0].mlp
    moe.eval()
    h = torch.randn(2, 16, 64)
    moe.dispatch = "dense"
    a = moe(h)
    moe.dispatch = "sparse"
    b = moe(h)
    assert torch.allclose(a, b, atol=1e-5)


def test_mla_rope_interleaved_equals_complex_form():
    from llm_in_practise_amd.ops.reference import apply_rope, rope_cos_sin
    x = torch.randn(10, 2, 8)
    cos, sin = rope_cos_sin(torch.arange(10), 8, 1e4)
    y = apply_rope(x, cos, sin, interleaved=True)
    xc = torch.view_as_complex(x.reshape(10, 2, 4, 2))
    f = torch.polar(torch.ones(10, 4), torch.outer(torch.arange(10).float(), 1 / 1e4 ** (torch.arange(0, 8, 2) / 8)))
    ref = torch.view_as_real(xc * f[:, None]).reshape(10, 2, 8)
    assert torch.allclose(y, ref, atol=1e-5)


@pytest.mark.parametrize("cls,args", [
    (L.MultiHeadAttention, (64, 8)),
    (L.GroupedQueryAttention, (64, 8, 2)),
    (L.MultiQueryAttention, (64, 8)),
    (L.LocalAttention, (64, 8, 3)),
])
def test_attention_variants(cls, args):
    m = cls(*args)
    x = torch.randn(2, 12, 64)
    assert m(x).shape == x.shape


def test_gqa_with_full_groups_equals_mha():
    torch.manual_seed(0)
    g = L.GroupedQueryAttention(64, 8, 8)
    m = L.MultiHeadAttention(64, 8)
    m.load_state_dict(g.state_dict())
    x = torch.randn(2, 10, 64)
    assert torch.allclose(g(x), m(x), atol=1e-6)


def test_local_attention_matches_loop():
    torch.manual_seed(0)
    m = L.LocalAttention(32, 4, 2)
    x = torch.randn(1, 9, 32)
    q = m.W_q(x).view(1, 9, 4, 8).transpose(1, 2)
    k = m.W_k(x).view(1, 9, 4, 8).transpose(1, 2)
    v = m.W_v(x).view(1, 9, 4, 8).transpose(1, 2)
    ctx = torch.zeros_like(q)
    for i in range(9):
        s, e = max(0, i - 2), min(9, i + 3)
        a = torch.softmax(q[:, :, i:i + 1] @ k[:, :, s:e].transpose(-1, -2) / math.sqrt(8), -1)
        ctx[:, :, i:i + 1] = a @ v[:, :, s:e]
    ref = m.W_o(ctx.transpose(1, 2).reshape(1, 9, 32))
    assert torch.allclose(m(x), ref, atol=1e-5)


def test_mla_returns_latent_cache():
    m = L.MultiHeadLatentAttention(64, 4, 32, 16)
    out, ckv = m(torch.randn(2, 7, 64))
    assert out.shape == (2, 7, 64) and ckv.shape == (2, 7, 32)


def test_blocks_and_stochastic_depth():
    x = torch.randn(2, 6, 32)
    mask = torch.triu(torch.ones(6, 6), 1) * float("-inf")
    assert L.ResiDualTransformerBlock(32, 4, 64)(x, attn_mask=mask).shape == x.shape
    assert L.ParallelTransformerBlock(32, 4, 64)(x, attn_mask=mask).shape == x.shape
    sd = L.StochasticDepth(0.5).eval()
    r = torch.randn_like(x)
    assert torch.equal(sd(x, r), x + r)
    blk = L.StochasticDepthBlock(32, 4, 64).eval()
    assert blk(x).shape == x.shape


def test_mha_module_matches_torch_nn():
    torch.manual_seed(0)
    ours = L.MultiheadAttention(32, 4, batch_first=True).eval()
    ref = nn.MultiheadAttention(32, 4, batch_first=True).eval()
    ref.load_state_dict(ours.state_dict())
    x = torch.randn(2, 9, 32)
    mask = torch.triu(torch.ones(9, 9), 1).bool()
    kpm = torch.zeros(2, 9, dtype=torch.bool)
    kpm[1, 7:] = True
    a = ours(x, x, x, attn_mask=mask, key_padding_mask=kpm)[0]
    b = ref(x, x, x, attn_mask=mask, key_padding_mask=kpm)[0]
    assert torch.allclose(a, b, atol=1e-5)


def test_fused_micro_batches_equal_mean_of_losses():
    """num_micro_batches=G (one pass) == mean of G separate micro-batch losses (CPU path)."""
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, seed=0)
    ids = torch.randint(0, 512, (4, 16))
    lab = ids.clone()
    lab[0, :10] = -100
    fused = m(ids, labels=lab, num_micro_batches=2).loss
    sep = (m(ids[:2], labels=lab[:2]).loss + m(ids[2:], labels=lab[2:]).loss) / 2
    assert torch.allclose(fused, sep, rtol=1e-5)


def test_gradient_checkpointing_kwargs_select_the_form(monkeypatch):
    """gradient_checkpointing_kwargs (HF API, Fine-Tuning/qwen3-8b-qlora-dist.py:162-163): use_reentrant
    selects torch's checkpoint form, ``policy`` the recompute policy; unknown keys raise; gradients match
    the un-checkpointed model in every form."""
    import torch.utils.checkpoint as tuc

    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    seen = []
    real = tuc.checkpoint

    def spy(fn, *a, use_reentrant=None, **k):
        seen.append(use_reentrant)
        return real(fn, *a, use_reentrant=use_reentrant, **k)

    monkeypatch.setattr(tuc, "checkpoint", spy)
    ids = torch.randint(0, 100, (2, 16))
    ref = None
    for kw in (None, {}, {"use_reentrant": False}, {"use_reentrant": True, "policy": "full"},
               {"use_reentrant": False, "policy": "selective"}):
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, seed=3)
        m.train()
        if kw is not None:
            m.gradient_checkpointing_enable(kw)
        seen.clear()
        m(ids, labels=ids).loss.backward()
        g = torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])
        if kw is None:
            ref = g
            assert seen == []
        else:
            assert seen and all(s == kw.get("use_reentrant", True) for s in seen), (kw, seen)
            assert torch.allclose(g, ref, atol=1e-5, rtol=1e-4)
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, seed=3)
    with pytest.raises(ValueError):
        m.gradient_checkpointing_enable({"preserve_rng": True})
