"""W4A16 int4 GEMMs (w4mm, gemm4w W4=2), 4-bit decode GEMV (NF4 + int4), GPTQ/AWQ on the GPU."""
import pytest
import torch

from llm_in_practise_amd.quant.int4 import int4_linear, quantize_rtn
from llm_in_practise_amd.quant.nf4 import dequantize_nf4, quantize_nf4

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-6)).item()


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("N,K", [(4096, 4096), (1024, 12288), (96, 256)])
def test_gemv_nf4_and_int4(native_ext, M, N, K):
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wq = quantize_nf4(torch.randn(N, K, device=DEV).to(torch.bfloat16), 64, True)
    y = native_ext.gemv_w4(x, wq.codes, wq.gemv_scales(), None, N, 64, None)
    assert rel(y, x.float() @ dequantize_nf4(wq, torch.float32).t()) < 1e-2
    w4 = quantize_rtn(torch.randn(N, K, device=DEV), 128, False)
    s, b = w4.gemv_tables()
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    y4 = native_ext.gemv_w4(x, w4.codes, s, b, N, 128, res)
    assert rel(y4, x.float() @ w4.dequantize().t() + res.float()) < 1e-2


@pytest.mark.parametrize("N,K,gs,sym", [(256, 512, 128, False), (384, 1024, 128, True), (96, 256, 64, False)])
def test_int4_linear_dispatch(native_ext, N, K, gs, sym):
    """Every row count through int4_linear's kernel choice — gemv_w4 (M <= 2), w4mm (3..32), w4g (33..64),
    gemm4w W4=2 (65..1023), the expansion + gemm4w prefill (>= 1024), the dequant fallback for shapes no kernel
    takes (N = 96) — against fp32, with residual."""
    torch.manual_seed(4)
    w = quantize_rtn(torch.randn(N, K, device=DEV), gs, sym)
    for M in (1, 2, 3, 8, 32, 33, 64, 100, 256, 300, 2048):
        x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        assert rel(int4_linear(x, w), x.float() @ w.dequantize().t()) < 1e-2, M
        assert rel(int4_linear(x, w, residual=res), x.float() @ w.dequantize().t() + res.float()) < 1e-2, M


@pytest.mark.parametrize("M", [33, 48, 64])
@pytest.mark.parametrize("N,K,gs", [(6144, 4096, 128), (4096, 12288, 128), (512, 1024, 256)])
def test_w4g_decode_batches(native_ext, M, N, K, gs):
    """The decode-batch W4A16 GEMM (w4g) at the Qwen3-8B q|k|v / down shapes and a 256-deep group: every
    K-slice count it may pick (1 = bf16 out + residual in-kernel, > 1 = fp32 partials + reduce) against fp32."""
    torch.manual_seed(6)
    w = quantize_rtn(torch.randn(N, K, device=DEV), gs, False)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    want = x.float() @ w.dequantize().t() + res.float()
    auto = native_ext.w4g_splits(M, N, K)
    for ks in sorted({1, 2, auto}):
        if (K // 128) % ks:
            continue
        y = native_ext.w4g(x, w.codes, w.w4mm_table(), N, gs, res, ks)
        assert y.shape == (M, N) and rel(y, want) < 1e-2, (ks, rel(y, want))


@pytest.mark.parametrize("N,K,gs,sym", [(256, 512, 128, False), (384, 1024, 64, True)])
def test_int4_dequant_kernel_matches_fp32(native_ext, N, K, gs, sym):
    """The HBM-speed int4 -> bf16 expansion (the W4A16 prefill form) against the fp32 dequantisation."""
    torch.manual_seed(5)
    w = quantize_rtn(torch.randn(N, K, device=DEV), gs, sym)
    s, b = w.gemv_tables()
    got = native_ext.int4_dequant(w.codes, s, b, N, K, gs)
    ref = w.dequantize()
    assert got.dtype == torch.bfloat16 and got.shape == (N, K)
    assert (got.float() - ref).abs().max() <= 1e-2 * ref.abs().max()


def test_awq_gptq_on_gpu_and_quantized_generation(native_ext):
    from llm_in_practise_amd.infer.generate import generate
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from llm_in_practise_amd.quant.awq import awq_quantize_model
    from llm_in_practise_amd.quant.eval import dataset_ppl
    from llm_in_practise_amd.quant.gptq import gptq_quantize_model
    calib = [torch.randint(0, 4096, (1, 128), device=DEV) for _ in range(4)]
    held = torch.randint(0, 4096, (1024,), device=DEV)
    base = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device=DEV, seed=0).eval()
    p0 = dataset_ppl(base, held)
    for fn in (awq_quantize_model, gptq_quantize_model):
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device=DEV, seed=0).eval()
        fn(m, calib)
        p = dataset_ppl(m, held)
        assert abs(p - p0) / p0 < 0.05, (fn.__name__, p, p0)
        out = generate(m, torch.randint(0, 4096, (2, 16), device=DEV), max_new_tokens=8)
        assert out.shape == (2, 24)


def test_nf4_decode_uses_gemv_and_matches_recompute(native_ext):
    from llm_in_practise_amd.infer.generate import generate
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from llm_in_practise_amd.peft.lora import quantize_model_nf4
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device=DEV, seed=0).eval()
    quantize_model_nf4(m)
    m.fuse_projections()
    p = torch.randint(0, 4096, (1, 40), device=DEV)
    out = generate(m, p, max_new_tokens=4)
    ids = p.clone()
    with torch.no_grad():
        for _ in range(4):
            ids = torch.cat([ids, m(ids).logits[:, -1].float().argmax(-1, keepdim=True)], 1)
    assert torch.equal(out[0, :42], ids[0, :42])
