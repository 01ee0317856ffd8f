"""W4A16 int4: formats round-trip, GPTQ beats RTN, AWQ folding is function-preserving, quantised
checkpoints reload to identical logits (CPU, fp32 references)."""
import torch
import torch.nn as nn

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.quant import awq as AWQ
from llm_in_practise_amd.quant.eval import dataset_ppl, self_ppl
from llm_in_practise_amd.quant.gptq import GPTQ, gptq_quantize_model
from llm_in_practise_amd.quant.int4 import (Int4Linear, from_awq, from_compressed_tensors, from_gptq, quantize_rtn,
                                            to_awq, to_compressed_tensors, to_gptq)
from llm_in_practise_amd.quant.io import load_quantized, save_quantized


def test_formats_roundtrip_exact():
    torch.manual_seed(0)
    for sym in (False, True):
        w = quantize_rtn(torch.randn(64, 256), 128, sym)
        for to, frm in ((to_compressed_tensors, lambda d: from_compressed_tensors(d, 128, sym)),
                        (to_gptq, lambda d: from_gptq(d, 128, sym)), (to_awq, lambda d: from_awq(d, 128))):
            r = frm(to(w))
            assert torch.equal(r.q(), w.q()) and torch.equal(r.zeros, w.zeros)
            assert torch.allclose(r.scales, w.scales, rtol=1e-2)
    d = to_gptq(quantize_rtn(torch.randn(16, 128), 128))
    assert d["qweight"].shape == (16, 16) and d["qzeros"].shape == (1, 2) and d["scales"].dtype == torch.float16


def test_rtn_dequant_error_bounded():
    w = torch.randn(32, 256)
    q = quantize_rtn(w, 128)
    err = (q.dequantize() - w).abs().view(32, 2, 128)
    span = w.view(32, 2, 128).amax(-1) - w.view(32, 2, 128).amin(-1)
    assert (err.amax(-1) <= span / 15 * 0.5 + 1e-5).all()


def test_gptq_beats_rtn_on_calibration_output():
    torch.manual_seed(0)
    lin = nn.Linear(256, 64, bias=False)
    x = torch.randn(2048, 256) @ torch.randn(256, 256) * 0.1      # correlated inputs
    g = GPTQ(lin)
    g.add_batch(x)
    qg = g.quantize(128, False, 0.01)
    qr = quantize_rtn(lin.weight.detach(), 128)
    ref = x @ lin.weight.t()
    eg = (x @ qg.dequantize().t() - ref).pow(2).mean()
    er = (x @ qr.dequantize().t() - ref).pow(2).mean()
    assert eg < er * 0.9


def _tiny():
    cfg = qwen3_config("qwen3-tiny", intermediate_size=256)
    return Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0).eval()


def test_awq_fold_preserves_function():
    torch.manual_seed(0)
    m = _tiny()
    ids = torch.randint(0, 512, (2, 16))
    y0 = m(ids).logits
    layer = m.model.layers[0]
    s = torch.rand(128) + 0.5
    AWQ._fold(layer.input_layernorm, [layer.self_attn.q_proj, layer.self_attn.k_proj, layer.self_attn.v_proj], s)
    s2 = torch.rand(256) + 0.5
    AWQ._fold(layer.mlp.up_proj, [layer.mlp.down_proj], s2)
    assert torch.allclose(m(ids).logits, y0, atol=1e-4)


def test_gptq_and_awq_models_and_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    calib = [torch.randint(0, 512, (1, 64)) for _ in range(4)]
    held = torch.randint(0, 512, (256,))
    base = _tiny()
    ppl0 = dataset_ppl(base, held)
    for algo in ("gptq", "awq"):
        m = _tiny()
        (gptq_quantize_model if algo == "gptq" else AWQ.awq_quantize_model)(m, calib)
        assert isinstance(m.model.layers[0].self_attn.q_proj, Int4Linear)
        ppl = dataset_ppl(m, held)
        assert abs(ppl - ppl0) / ppl0 < 0.05                 # random-init model: tiny degradation
        for fmt in ("compressed-tensors", "gptq", "awq"):
            d = str(tmp_path / f"{algo}-{fmt}")
            save_quantized(m, d, fmt)
            r = load_quantized(d)
            ids = torch.randint(0, 512, (1, 12))
            assert torch.allclose(r(ids).logits.float(), m(ids).logits.float(), atol=2e-2), (algo, fmt)
    assert self_ppl(base, [torch.randint(0, 512, (8,))], max_new_tokens=8) > 1.0
