"""CPU tests: NF4 format, LoRA / QLoRA adapters (PEFT-compatible IO, merge), optimizers."""
import json
import os

import pytest
import torch

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.peft.lora import (LoraConfig, LoraLayer, PeftModel, get_peft_model,
                                           quantize_model_nf4)
from llm_in_practise_amd.quant.nf4 import (NF4_CODE, concat_nf4, create_dynamic_map, dequantize_nf4,
                                           quantize_nf4)


def test_nf4_codebook_roundtrip_exact():
    # every code value times a block absmax must round-trip exactly through quantisation
    code = torch.tensor(NF4_CODE)
    w = code.repeat(8).view(2, 64) * 3.0
    q = quantize_nf4(w, 64, double_quant=False)
    assert torch.allclose(dequantize_nf4(q, torch.float32), w)
    # nibble packing: first element in the HIGH nibble
    assert (q.codes[0, 0] >> 4).item() == 0 and (q.codes[0, 0] & 15).item() == 1


def test_nf4_error_and_double_quant():
    torch.manual_seed(0)
    w = torch.randn(256, 512)
    q1 = quantize_nf4(w, 64, double_quant=False)
    q2 = quantize_nf4(w, 64, double_quant=True)
    e1 = (dequantize_nf4(q1, torch.float32) - w).pow(2).mean().sqrt() / w.std()
    e2 = (dequantize_nf4(q2, torch.float32) - w).pow(2).mean().sqrt() / w.std()
    assert e1 < 0.12 and e2 < 0.125 and e2 >= e1 * 0.99
    assert q2.qabsmax.dtype == torch.uint8 and q2.absmax2.numel() == 256 * 512 // 64 // 256
    assert q2.nbytes() < q1.nbytes()


def test_dynamic_maps():
    s, u = create_dynamic_map(True), create_dynamic_map(False)
    assert s.numel() == u.numel() == 256
    assert s.min() < 0 and u.min() == 0 and s.max() == 1.0 and u.max() == 1.0
    assert torch.all(s[1:] >= s[:-1]) and torch.all(u[1:] >= u[:-1])


def test_concat_nf4_is_exact():
    torch.manual_seed(0)
    ws = [torch.randn(n, 256) for n in (256, 128, 64)]
    qs = [quantize_nf4(w, 64) for w in ws]
    fused = concat_nf4(qs)
    ref = torch.cat([dequantize_nf4(q, torch.float32) for q in qs])
    assert torch.equal(dequantize_nf4(fused, torch.float32), ref)


def _tiny(dtype=torch.float32, seed=0):
    cfg = qwen3_config("qwen3-tiny")
    return cfg, Qwen3ForCausalLM.from_config(cfg, dtype=dtype, seed=seed)


def test_lora_injection_counts_match_peft():
    cfg, m = _tiny()
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, target_modules=["q_proj", "v_proj"]))
    t, _ = pm.get_nb_trainable_parameters()
    h, L = cfg.hidden_size, cfg.num_hidden_layers
    q_out, v_out = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
    assert t == L * (8 * h + 8 * q_out + 8 * h + 8 * v_out)
    assert isinstance(m.model.layers[0].self_attn.q_proj, LoraLayer)
    assert not isinstance(m.model.layers[0].self_attn.k_proj, LoraLayer)


def test_qwen3_8b_lora_param_count_matches_reference():
    """Qwen3-8B r8 q,v -> 3,833,856 trainable; E1 r16 qkvo -> 15,335,424."""
    cfg = qwen3_config("qwen3-8b")
    h, L, qo, vo = cfg.hidden_size, cfg.num_hidden_layers, 32 * 128, 8 * 128
    assert L * 8 * ((h + qo) + (h + vo)) == 3_833_856
    assert L * 16 * ((h + qo) + 2 * (h + vo) + (qo + h)) == 15_335_424


def test_adapter_save_load_roundtrip(tmp_path):
    _, m = _tiny()
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"]))
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_B" in n:
                p.normal_()
    pm.save_pretrained(str(tmp_path))
    keys = json.load(open(tmp_path / "adapter_config.json"))
    assert keys["r"] == 4 and sorted(keys["target_modules"]) == ["q_proj", "v_proj"]
    from safetensors.torch import load_file
    sd = load_file(str(tmp_path / "adapter_model.safetensors"))
    assert "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight" in sd
    _, m2 = _tiny()
    pm2 = PeftModel.from_pretrained(m2, str(tmp_path))
    for (n1, p1), (n2, p2) in zip(pm.named_parameters(), pm2.named_parameters()):
        if "lora_" in n1:
            assert torch.equal(p1, p2)
    ids = torch.randint(0, 512, (1, 12))
    pm.eval()
    assert torch.allclose(pm(ids).logits, pm2(ids).logits, atol=1e-5)


@pytest.mark.parametrize("quant", [False, True])
def test_merge_and_unload_matches_adapter(quant):
    _, m = _tiny()
    if quant:
        quantize_model_nf4(m, compute_dtype=torch.float32)
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"]))
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.1)
    pm.eval()
    ids = torch.randint(0, 512, (2, 10))
    before = pm(ids).logits
    merged = pm.merge_and_unload()
    after = merged(ids).logits
    assert torch.allclose(before, after, atol=1e-4)


def test_fused_projections_equal_unfused():
    _, m = _tiny()
    quantize_model_nf4(m, compute_dtype=torch.float32)
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"]))
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.1)
    pm.eval()
    ids = torch.randint(0, 512, (2, 16))
    a = pm(ids).logits
    m.fuse_projections()
    b = pm(ids).logits
    assert torch.allclose(a, b, atol=1e-5)


def test_qlora_training_loss_decreases():
    from llm_in_practise_amd.optim.adamw import build_optimizer
    _, m = _tiny()
    quantize_model_nf4(m, compute_dtype=torch.float32)
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    m.fuse_projections()
    opt = build_optimizer("paged_adamw_8bit", [p for p in pm.parameters() if p.requires_grad], 3e-3)
    ids = torch.randint(0, 512, (4, 32))
    losses = []
    for _ in range(25):
        out = pm(ids, labels=ids)
        out.loss.backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad()
        losses.append(out.loss.item())
    assert losses[-1] < losses[0] - 0.3


def test_ga_fused_pass_equals_sequential():
    _, m = _tiny()
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, target_modules=["q_proj", "v_proj"]))
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_B" in n:
                p.normal_(0, 0.1)
    ids = torch.randint(0, 512, (4, 16))
    labels = ids.clone()
    labels[0, 10:] = -100                       # unequal valid counts per micro-batch
    grads = []
    for fused in (False, True):
        pm.zero_grad()
        if fused:
            pm(ids, labels=labels, num_micro_batches=2).loss.backward()
        else:
            for g in range(2):
                (pm(ids[2 * g:2 * g + 2], labels=labels[2 * g:2 * g + 2]).loss / 2).backward()
        grads.append([p.grad.clone() for p in pm.parameters() if p.requires_grad])
    for a, b in zip(*grads):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-4)


def test_checkpoint_replays_dropout_key_stream():
    """ops.linear.checkpoint restores the host dropout-key stream for the recompute, so the
    backward sees the forward's key; the live stream advances exactly once per real forward."""
    from llm_in_practise_amd.ops import linear as L
    L.seed_dropout(7)
    seen = []

    def fn(x):
        k = L.next_dropout_key()
        seen.append(k)
        return x * x * float(k % 997 + 1)      # saves x: backward must recompute

    x = torch.ones(3, requires_grad=True)
    y = L.checkpoint(fn, x)
    after_fwd = L._KEY[0]
    y.sum().backward()
    assert len(seen) == 2 and seen[0] == seen[1]              # recompute drew the same key
    assert L._KEY[0] == after_fwd                             # stream not advanced by the recompute
    assert torch.allclose(x.grad, torch.full((3,), 2.0 * float(seen[0] % 997 + 1)))


def test_checkpointed_qwen3_lora_grads_match_including_layer0():
    """Gradient checkpointing (reentrant default) gives the same LoRA gradients as the plain pass —
    including layer 0, whose input (the frozen embedding's output) does not require grad (the
    reentrant form needs the input marked, as HF's enable_input_require_grads() does)."""
    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model
    grads = []
    for ck in (False, True):
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.float32, device="cpu", seed=3)
        pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
        for n, p in pm.named_parameters():
            if p.requires_grad and "lora_B" in n:
                torch.nn.init.normal_(p, std=0.02, generator=torch.Generator().manual_seed(len(n)))
        if ck:
            pm.gradient_checkpointing_enable()
        pm.train()
        ids = torch.randint(0, 100, (2, 16), generator=torch.Generator().manual_seed(1))
        pm(ids, labels=ids).loss.backward()
        grads.append({n: p.grad.clone() for n, p in pm.named_parameters() if p.requires_grad and p.grad is not None})
    assert grads[0].keys() == grads[1].keys() and any(".0." in n for n in grads[1])
    for n in grads[0]:
        assert torch.allclose(grads[0][n], grads[1][n], rtol=1e-4, atol=1e-6), n
