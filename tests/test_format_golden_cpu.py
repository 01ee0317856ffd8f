"""Format parity pinned to golden bytes / layouts derived from the published specs (the libraries
themselves — bitsandbytes, peft, deepspeed — are not importable here, so these tests hold the
format down independently of our own reader/writer pairs):

* NF4 (QLoRA paper, Dettmers et al. 2023, Appendix E; bitsandbytes ``kQuantizeBlockwise`` 4-bit):
  the 16-value code table, nearest-code index per element of ``x / absmax(block of 64)``, two
  indices per byte with the FIRST element in the HIGH nibble, fp32 absmax per block.
* PEFT LoRA adapters (``peft.PeftModel.save_pretrained``): ``adapter_model.safetensors`` keys
  ``base_model.model.<module path>.lora_A.weight`` [r, in] / ``.lora_B.weight`` [out, r] and an
  ``adapter_config.json`` with ``peft_type: LORA``, ``r``, ``lora_alpha``, ``lora_dropout``,
  ``target_modules``, ``bias``, ``task_type``.
* DeepSpeed ZeRO checkpoints (``engine.save_checkpoint``): ``<dir>/latest`` holding the tag,
  ``<dir>/<tag>/mp_rank_00_model_states.pt`` and one ``zero_pp_rank_<r>_mp_rank_00_optim_states.pt``
  per data-parallel rank.
"""
import json
import os

import torch

from llm_in_practise_amd.quant.nf4 import NF4_CODE, dequantize_nf4, quantize_nf4

# QLoRA paper / bitsandbytes NF4 table (float32 literals as published)
PUBLISHED_NF4 = [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
                 -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
                 0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
                 0.7229568362236023, 1.0]


def test_nf4_table_is_the_published_one():
    assert NF4_CODE == PUBLISHED_NF4


def test_nf4_golden_bytes():
    # one 64-element block whose absmax is 2.0; element i = 2.0 * code[i % 16] (exactly representable)
    # -> indices 0,1,...,15 repeated; bytes = (idx[2j] << 4) | idx[2j+1] = 0x01, 0x23, ..., 0xEF
    w = torch.tensor([2.0 * PUBLISHED_NF4[i % 16] for i in range(64)]).view(1, 64)
    q = quantize_nf4(w, 64, double_quant=False)
    golden = bytes([0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF] * 4)
    assert bytes(q.codes.flatten().tolist()) == golden
    assert q.absmax.tolist() == [2.0]
    # a value between two codes goes to the nearer one: 0.5 * (code[8] + code[9]) + eps -> 9
    mid = 0.5 * (PUBLISHED_NF4[8] + PUBLISHED_NF4[9])
    w2 = torch.full((1, 64), 0.0)
    w2[0, 0] = 1.0                                   # absmax 1.0
    w2[0, 1] = mid + 1e-4                            # -> index 9
    w2[0, 2] = mid - 1e-4                            # -> index 8
    w2[0, 3] = -1.0                                  # -> index 0
    q2 = quantize_nf4(w2, 64, double_quant=False)
    b = q2.codes.flatten().tolist()
    assert b[0] == (15 << 4) | 9 and b[1] == (8 << 4) | 0 and b[2] == (7 << 4) | 7   # zeros -> index 7
    assert torch.allclose(dequantize_nf4(q2, torch.float32)[0, :4],
                          torch.tensor([1.0, PUBLISHED_NF4[9], PUBLISHED_NF4[8], -1.0]))


def test_peft_adapter_layout(tmp_path):
    from safetensors import safe_open

    from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model
    cfg = qwen3_config("qwen3-tiny")
    m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0)
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["q_proj", "v_proj"]))
    pm.save_pretrained(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == ["adapter_config.json", "adapter_model.safetensors"]
    with open(tmp_path / "adapter_config.json") as f:
        c = json.load(f)
    assert c["peft_type"] == "LORA" and c["task_type"] == "CAUSAL_LM" and c["r"] == 8 and c["lora_alpha"] == 16
    assert abs(c["lora_dropout"] - 0.05) < 1e-9 and c["bias"] == "none"
    assert sorted(c["target_modules"]) == ["q_proj", "v_proj"]
    hd = cfg.head_dim
    want = {}
    for i in range(cfg.num_hidden_layers):
        for proj, out in (("q_proj", cfg.num_attention_heads * hd), ("v_proj", cfg.num_key_value_heads * hd)):
            pre = f"base_model.model.model.layers.{i}.self_attn.{proj}"
            want[pre + ".lora_A.weight"] = [8, cfg.hidden_size]
            want[pre + ".lora_B.weight"] = [out, 8]
    with safe_open(str(tmp_path / "adapter_model.safetensors"), "pt") as f:
        got = {k: list(f.get_slice(k).get_shape()) for k in f.keys()}
    assert got == want


def test_deepspeed_zero_checkpoint_layout(tmp_path):
    from llm_in_practise_amd.parallel.zero import ZeroEngine
    net = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 2))
    eng = ZeroEngine(net, {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 1,
                           "zero_optimization": {"stage": 2}, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}})
    loss = eng(torch.randn(2, 8)).pow(2).mean()
    eng.backward(loss)
    eng.step()
    eng.save_checkpoint(str(tmp_path))
    tag = open(tmp_path / "latest").read().strip()
    assert tag == "global_step1"
    assert sorted(os.listdir(tmp_path / tag)) == ["mp_rank_00_model_states.pt", "zero_pp_rank_0_mp_rank_00_optim_states.pt"]
    ms = torch.load(tmp_path / tag / "mp_rank_00_model_states.pt", weights_only=True)
    assert "module" in ms and ms["global_steps"] == 1
