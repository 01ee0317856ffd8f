"""Decode-attention and sampler kernels vs the PyTorch references (fp32)."""
import math

import pytest
import torch

from llm_in_practise_amd.ops.decode import decode_attention_reference, sample_reference

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (8, 8, 64), (40, 8, 128), (16, 2, 64)])
@pytest.mark.parametrize("lens", [[1, 300, 4096, 129], [77]])
def test_decode_attention_kernel(native_ext, hq, hkv, d, lens):
    torch.manual_seed(0)
    B, Smax = len(lens), 4096
    kc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    q = torch.randn(B, hq * d, device=DEV).to(torch.bfloat16)
    L = torch.tensor(lens, device=DEV, dtype=torch.int32)
    o = native_ext.decode_attention(q, kc, vc, L, hq, hkv, d, max(lens), 1 / math.sqrt(d))
    r = decode_attention_reference(q.float(), kc.float(), vc.float(), L, hq, hkv, d)
    assert (o.float() - r).abs().max().item() < 2e-2


def test_sampler_greedy_and_topk1(native_ext):
    torch.manual_seed(0)
    x = torch.randn(8, 151936, device=DEV)
    g = x.argmax(-1)
    assert torch.equal(native_ext.sample(x, None, 0.0, 0, 1.0, 1.0, 1), g)
    assert torch.equal(native_ext.sample(x, None, 0.7, 1, 1.0, 1.0, 2), g)
    assert torch.equal(native_ext.sample(x.to(torch.bfloat16), None, 0.0, 0, 1.0, 1.0, 3),
                       x.to(torch.bfloat16).float().argmax(-1))
    assert torch.equal(native_ext.sample(x, None, 1.0, 0, 1e-6, 1.0, 4), g)


def test_sampler_penalty_matches_reference(native_ext):
    torch.manual_seed(1)
    x = torch.randn(4, 1000, device=DEV)
    hist = torch.randint(0, 1000, (4, 64), device=DEV, dtype=torch.int32)
    hist[:, 50:] = -1
    hist[:, 10] = hist[:, 11]           # duplicates
    want = sample_reference(x, hist, 0.0, penalty=1.3)
    assert torch.equal(native_ext.sample(x, hist, 0.0, 0, 1.0, 1.3, 5), want)


def test_sampler_distribution_top_p(native_ext):
    # probabilities 0.5/0.3/0.15/0.05; top_p 0.7 keeps {0,1} renormalised to 0.625/0.375
    p = torch.tensor([0.5, 0.3, 0.15, 0.05], device=DEV)
    x = torch.log(p)[None].repeat(20000, 1).contiguous()
    s = native_ext.sample(x, None, 1.0, 0, 0.7, 1.0, 12345)
    counts = torch.bincount(s, minlength=4).float() / s.numel()
    assert counts[2] == 0 and counts[3] == 0
    assert abs(counts[0].item() - 0.625) < 0.02
    s2 = native_ext.sample(x, None, 1.0, 3, 1.0, 1.0, 777)   # top-k 3
    c2 = torch.bincount(s2, minlength=4).float() / s2.numel()
    assert c2[3] == 0 and abs(c2[0].item() - 0.5 / 0.95) < 0.02


def test_generate_qwen3_gpu_kv_cache_matches_recompute(native_ext):
    from llm_in_practise_amd.infer.generate import generate
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device=DEV, seed=0).eval()
    p = torch.randint(0, 4096, (1, 33), device=DEV)
    out = generate(m, p, max_new_tokens=8)
    ids = p.clone()
    with torch.no_grad():
        for _ in range(8):
            ids = torch.cat([ids, m(ids).logits[:, -1].float().argmax(-1, keepdim=True)], 1)
    # bf16 rounding can flip near-ties late in the sequence; the first tokens must agree
    assert torch.equal(out[0, :37], ids[0, :37])


@pytest.mark.parametrize("B,max_len", [(64, 4096), (1, 1024), (7, 3000)])
def test_decode_attention_split_plans(native_ext, B, max_len):
    """Batch sizes that select different split plans (1 split per head up to 64-key chunks)."""
    torch.manual_seed(B)
    hq, hkv, d, Smax = 32, 8, 128, 4096
    kc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    q = torch.randn(B, hq * d, device=DEV).to(torch.bfloat16)
    L = torch.randint(1, max_len + 1, (B,), device=DEV, dtype=torch.int32)
    L[0] = max_len
    o = native_ext.decode_attention(q, kc, vc, L, hq, hkv, d, max_len, 1 / math.sqrt(d))
    r = decode_attention_reference(q.float(), kc.float(), vc.float(), L, hq, hkv, d)
    assert (o.float() - r).abs().max().item() < 2e-2


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (8, 8, 64), (40, 8, 128), (16, 1, 64), (64, 4, 128)])
@pytest.mark.parametrize("pos", [[0, 299, 4095, 128], [76], [31, 32, 33, 1000, 1023, 1024, 5, 64]])
def test_decode_attention_append_kernel(native_ext, hq, hkv, d, pos):
    """MFMA decode kernel with the fused KV append: q/k/v are row-strided views of one fused
    qkv projection output; the new rows must land in the caches at pos and take part in the
    attention; no other cache row may change."""
    torch.manual_seed(len(pos) + hq)
    B, Smax = len(pos), 4096
    kc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, Smax, hkv * d, device=DEV).to(torch.bfloat16)
    qkv = torch.randn(B, (hq + 2 * hkv) * d, device=DEV).to(torch.bfloat16)
    q, k, v = qkv[:, :hq * d], qkv[:, hq * d:(hq + hkv) * d], qkv[:, (hq + hkv) * d:]
    P = torch.tensor(pos, device=DEV, dtype=torch.long)
    kc0, vc0 = kc.clone(), vc.clone()
    o = native_ext.decode_attention_append(q, k, v, kc, vc, P, hq, hkv, d, max(pos) + 1, 1 / math.sqrt(d))
    rows = torch.arange(B, device=DEV)
    kc0[rows, P] = k
    vc0[rows, P] = v
    assert torch.equal(kc, kc0) and torch.equal(vc, vc0)
    r = decode_attention_reference(q.float(), kc0.float(), vc0.float(), (P + 1).int(), hq, hkv, d)
    assert (o.float() - r).abs().max().item() < 2e-2


@pytest.mark.parametrize("B,max_len", [(256, 1024), (64, 4096), (1, 1024), (7, 3000)])
def test_decode_attention_append_split_plans(native_ext, B, max_len):
    torch.manual_seed(B)
    hq, hkv, d = 32, 8, 128
    kc = torch.randn(B, max_len, hkv * d, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, max_len, hkv * d, device=DEV).to(torch.bfloat16)
    q = torch.randn(B, hq * d, device=DEV).to(torch.bfloat16)
    k = torch.randn(B, hkv * d, device=DEV).to(torch.bfloat16)
    v = torch.randn(B, hkv * d, device=DEV).to(torch.bfloat16)
    P = torch.randint(0, max_len, (B,), device=DEV)
    P[0] = max_len - 1
    o = native_ext.decode_attention_append(q, k, v, kc, vc, P, hq, hkv, d, max_len, 1 / math.sqrt(d))
    r = decode_attention_reference(q.float(), kc.float(), vc.float(), (P + 1).int(), hq, hkv, d)
    assert (o.float() - r).abs().max().item() < 2e-2


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 12288), (272, 192)])
def test_gemm_skinny_matches_fp32(native_ext, M, N, K):
    """Decode-shaped split-K GEMM (+ residual) vs fp32, incl. N not a multiple of the 128-row block."""
    torch.manual_seed(M)
    w = (torch.randn(N, K, device=DEV) * 0.02).to(torch.bfloat16)
    xb = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    x = xb[:, :K]                                   # row-strided input
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = native_ext.gemm_skinny(x, w, None)
    assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    y = native_ext.gemm_skinny(x, w, res)
    want = ref + res.float()
    assert ((y.float() - want).abs().max() / want.abs().max()).item() < 1e-2
