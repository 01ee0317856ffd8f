"""Trainer + ZeRO engine on the GPU (native kernels): QLoRA qwen3-small trains, checkpoints,
resumes bit-exactly; ZeRO-3 single-rank path runs the fused kernels."""
import os

import pytest
import torch

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4
from llm_in_practise_amd.train.data import SyntheticLMDataset
from llm_in_practise_amd.train.trainer import Trainer, TrainingArguments

pytestmark = pytest.mark.gpu


def _qlora(seed=0):
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device="cuda", seed=seed)
    quantize_model_nf4(m)
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.1, target_modules=["q_proj", "v_proj"]))
    pm.fuse_projections()
    return pm


class _Collate:
    def __call__(self, rows):
        ids = torch.tensor([r["input_ids"] for r in rows])
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "labels": ids.clone()}


def _args(out, **kw):
    a = dict(output_dir=str(out), per_device_train_batch_size=2, gradient_accumulation_steps=2, max_steps=6,
             learning_rate=1e-3, logging_steps=1, save_steps=3, save_total_limit=2, optim="paged_adamw_8bit",
             bf16=True, seed=3)
    a.update(kw)
    return TrainingArguments(**a)


def test_qlora_trainer_gpu_resume_exact(tmp_path, native_ext, monkeypatch):
    monkeypatch.setenv("LIPA_DETERMINISTIC", "1")     # fixed-order LoRA grad sums (no fp32 atomics)
    torch.manual_seed(0)
    ds = SyntheticLMDataset(4096, 128, 16, seed=1)
    full = _qlora()
    tr = Trainer(full, _args(tmp_path / "a"), train_dataset=ds, data_collator=_Collate())
    out = tr.train()
    losses = [h["loss"] for h in tr.state.log_history if "loss" in h]
    assert all(l == l for l in losses) and out.global_step == 6
    want = {k: v.clone() for k, v in full.adapter_state_dict().items()}

    os.environ["FAULT_INJECT"] = "0:4:raise"
    try:
        part = _qlora()
        with pytest.raises(Exception):
            Trainer(part, _args(tmp_path / "b"), train_dataset=ds, data_collator=_Collate()).train()
    finally:
        os.environ.pop("FAULT_INJECT")
    res = _qlora()
    tr2 = Trainer(res, _args(tmp_path / "b"), train_dataset=ds, data_collator=_Collate())
    tr2.train(resume_from_checkpoint=str(tmp_path / "b" / "checkpoint-3"))
    got = res.adapter_state_dict()
    for k in want:
        assert torch.allclose(got[k], want[k], atol=1e-6), k


def test_zero3_single_rank_gpu(tmp_path, native_ext):
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=torch.bfloat16, device="cuda", seed=0)
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))
    ds = SyntheticLMDataset(512, 64, 8, seed=2)
    cfg = {"bf16": {"enabled": True}, "zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0},
           "gradient_accumulation_steps": "auto", "train_micro_batch_size_per_gpu": "auto",
           "gradient_clipping": 1.0}
    tr = Trainer(pm, _args(tmp_path, optim="adamw_torch", deepspeed=cfg, max_steps=4, save_steps=2),
                 train_dataset=ds, data_collator=_Collate())
    out = tr.train()
    assert out.global_step == 4 and out.training_loss == out.training_loss
    assert os.path.isdir(tmp_path / "checkpoint-4" / "global_step4")


@pytest.mark.parametrize("targets", [["q_proj", "v_proj"], ["q_proj", "k_proj", "v_proj", "o_proj"]])
@pytest.mark.parametrize("kw", [{}, {"use_reentrant": False}, {"policy": "full"},
                                {"use_reentrant": False, "policy": "full"}])
def test_grad_ckpt_lora_dropout_same_gradients(native_ext, monkeypatch, targets, kw):
    """Gradient checkpointing must replay the exact LoRA dropout masks of the forward: LoRA
    gradients with and without checkpointing agree at dropout 0.1 (Fine-Tuning/qwen3-8b-lora.py:123),
    for both torch checkpoint forms (use_reentrant, qwen3-8b-qlora-dist.py:162-163) and both recompute
    policies (selective: the GEMM outputs of the first forward replayed; full: the whole layer again)."""
    import llm_in_practise_amd.ops.linear as L
    from llm_in_practise_amd.ops.linear import seed_dropout
    monkeypatch.setenv("LIPA_DETERMINISTIC", "1")
    grads = []
    for ck in (False, True):
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device="cuda", seed=5)
        quantize_model_nf4(m)
        pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.1, target_modules=targets))
        pm.fuse_projections()
        if ck:
            pm.gradient_checkpointing_enable(kw)
        pm.train()
        for n, p in pm.named_parameters():       # non-zero B so dA carries the mask too
            if p.requires_grad and "lora_B" in n:
                torch.nn.init.normal_(p, std=0.02, generator=torch.Generator(device="cuda").manual_seed(hash(n) % 1000))
        seed_dropout(123)
        ids = torch.randint(0, 1000, (2, 128), device="cuda", generator=torch.Generator(device="cuda").manual_seed(9))
        out = pm(ids, labels=ids)
        out.loss.backward()
        grads.append({n: p.grad.detach().float().clone() for n, p in pm.named_parameters() if p.requires_grad})
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        assert (a - b).norm() <= 2e-3 * a.norm() + 1e-6, n


def test_lora_pair_kernels_match_single_branch_path(native_ext, monkeypatch):
    """q_proj + v_proj through the two-branch kernels (one x / dx pass) give the same loss and
    LoRA gradients as the per-adapter kernels, dropout 0.1 included (same counter-RNG keys)."""
    from llm_in_practise_amd.ops.linear import seed_dropout
    torch.manual_seed(0)
    ids = torch.randint(0, 1000, (2, 64), device="cuda")
    res = {}
    import llm_in_practise_amd.ops.linear as L
    for mode in ("0", "1"):
        monkeypatch.setattr(L, "_PAIR", mode == "1")
        pm = _qlora(seed=0)
        pm.train()
        seed_dropout(42)
        out = pm(input_ids=ids, labels=ids)
        out.loss.backward()
        res[mode] = (out.loss.item(), {n: p.grad.float().clone() for n, p in pm.named_parameters() if p.requires_grad})
    (l0, g0), (l1, g1) = res["0"], res["1"]
    assert abs(l0 - l1) < 1e-3 * abs(l0)
    for n in g0:
        err = (g0[n] - g1[n]).norm() / g0[n].norm().clamp(min=1e-12)
        assert err < 2e-2, (n, float(err))


@pytest.mark.parametrize("targets,r,quant", [(["q_proj", "v_proj"], 8, True), (["q_proj", "k_proj", "v_proj", "o_proj"], 16, True),
                                             (["q_proj", "k_proj", "v_proj", "o_proj"], 16, False)])
def test_lora_dx_as_gemm_c_matches_read_modify_write(native_ext, monkeypatch, targets, r, quant):
    """At training sizes (M >= 256) the adapters' masked dx terms ride inside the dX GEMM (gemm4w_loradx, from
    the stored keep bits) and dA / dB run in the pair / multi launches; the loss and LoRA gradients match the
    per-adapter read-modify-write path that LIPA_DETERMINISTIC=1 selects (lora_acc per adapter, dropout masks
    regenerated from the keys), dropout 0.1 included."""
    import llm_in_practise_amd.ops.linear as L
    torch.manual_seed(0)
    ids = torch.randint(0, 1000, (2, 256), device="cuda")
    res = {}
    for mode in (False, True):
        monkeypatch.setenv("LIPA_DETERMINISTIC", "0" if mode else "1")
        m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-small"), dtype=torch.bfloat16, device="cuda", seed=0)
        if quant:
            quantize_model_nf4(m)
        pm = get_peft_model(m, LoraConfig(r=r, lora_alpha=2 * r, lora_dropout=0.1, target_modules=targets))
        pm.fuse_projections()
        pm.train()
        for n, p in pm.named_parameters():       # non-zero B so the dx / dA terms carry the masks
            if p.requires_grad and "lora_B" in n:
                torch.nn.init.normal_(p, std=0.02, generator=torch.Generator(device="cuda").manual_seed(hash(n) % 1000))
        L.seed_dropout(42)
        out = pm(input_ids=ids, labels=ids)
        out.loss.backward()
        res[mode] = (out.loss.item(), {n: p.grad.float().clone() for n, p in pm.named_parameters() if p.requires_grad})
    (l0, g0), (l1, g1) = res[False], res[True]
    assert abs(l0 - l1) < 1e-3 * abs(l0)
    for n in g0:
        err = (g0[n] - g1[n]).norm() / g0[n].norm().clamp(min=1e-12)
        assert err < 2e-2, (n, float(err))
