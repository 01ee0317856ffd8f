"""Trainer on CPU: loss decreases, HF checkpoint layout + rotation, bit-exact resume after an
injected fault, fused-GA == sequential GA, DDP world-2 (gloo) == single process."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model
from llm_in_practise_amd.train.data import DataCollatorForLanguageModeling, SyntheticLMDataset
from llm_in_practise_amd.train.trainer import Trainer, TrainingArguments
from llm_in_practise_amd.utils.faults import InjectedFault


def _model(seed=0, dtype=torch.float32):
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny"), dtype=dtype, seed=seed)
    return get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=["q_proj", "v_proj"]))


class _PadCollator:
    def __call__(self, rows):
        ids = torch.tensor([r["input_ids"] for r in rows])
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "labels": ids.clone()}


def _args(tmp, **kw):
    base = dict(output_dir=str(tmp), per_device_train_batch_size=2, gradient_accumulation_steps=2,
                max_steps=6, learning_rate=1e-2, logging_steps=1, save_steps=3, save_total_limit=2,
                optim="adamw_torch", seed=7)
    base.update(kw)
    return TrainingArguments(**base)


def _adapter(model):
    return {k: v.clone() for k, v in model.adapter_state_dict().items()}


def test_trainer_loss_decreases_and_layout(tmp_path):
    ds = SyntheticLMDataset(512, 32, 8, seed=1)
    m = _model()
    tr = Trainer(m, _args(tmp_path, max_steps=12, save_steps=4), train_dataset=ds, data_collator=_PadCollator())
    out = tr.train()
    hist = [h["loss"] for h in tr.state.log_history if "loss" in h]
    assert hist[-1] < hist[0]
    cks = sorted(os.listdir(tmp_path))
    assert cks == ["checkpoint-12", "checkpoint-8"]                # save_total_limit=2 rotation
    files = set(os.listdir(tmp_path / "checkpoint-12"))
    assert {"adapter_model.safetensors", "adapter_config.json", "optimizer.pt", "scheduler.pt", "rng_state.pth",
            "trainer_state.json", "training_args.bin"} <= files
    st = json.load(open(tmp_path / "checkpoint-12" / "trainer_state.json"))
    assert st["global_step"] == 12
    args = torch.load(tmp_path / "checkpoint-12" / "training_args.bin", weights_only=True)
    assert args["save_total_limit"] == 2
    tr.save_metrics("train", out.metrics)
    assert os.path.exists(tmp_path / "train_results.json") and os.path.exists(tmp_path / "all_results.json")


def test_resume_is_bit_exact_after_injected_fault(tmp_path, monkeypatch):
    ds = SyntheticLMDataset(512, 32, 12, seed=2)
    full = _model()
    Trainer(full, _args(tmp_path / "a"), train_dataset=ds, data_collator=_PadCollator()).train()
    want = _adapter(full)

    monkeypatch.setenv("FAULT_INJECT", "0:5:raise")
    crashed = _model()
    tr = Trainer(crashed, _args(tmp_path / "b"), train_dataset=ds, data_collator=_PadCollator())
    with pytest.raises(InjectedFault):
        tr.train()
    d = tr.save_interrupted()
    assert os.path.exists(os.path.join(d, "adapter_model.safetensors"))
    monkeypatch.delenv("FAULT_INJECT")
    resumed = _model()
    with torch.no_grad():                             # scramble adapters: resume must restore them
        for n, p in resumed.named_parameters():
            if "lora_" in n:
                p.normal_()
    tr2 = Trainer(resumed, _args(tmp_path / "b"), train_dataset=ds, data_collator=_PadCollator())
    tr2.train(resume_from_checkpoint=True)
    got = _adapter(resumed)
    for k in want:
        assert torch.equal(got[k], want[k]), k


def test_fused_ga_matches_sequential(tmp_path):
    ds = SyntheticLMDataset(512, 32, 8, seed=3)
    a, b = _model(), _model()
    Trainer(a, _args(tmp_path / "a", ga_fusion=True, save_steps=0, max_steps=3), train_dataset=ds,
            data_collator=_PadCollator()).train()
    Trainer(b, _args(tmp_path / "b", ga_fusion=False, save_steps=0, max_steps=3), train_dataset=ds,
            data_collator=_PadCollator()).train()
    wa, wb = _adapter(a), _adapter(b)
    for k in wa:
        assert torch.allclose(wa[k], wb[k], atol=1e-5), k


def _ddp_worker(rank, world, port, out, ds_cfg):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    ds = SyntheticLMDataset(512, 32, 8, seed=4)
    m = _model()
    args = _args(out + "_dir", per_device_train_batch_size=1, save_steps=0, max_steps=3, deepspeed=ds_cfg)
    Trainer(m, args, train_dataset=ds, data_collator=_PadCollator()).train()
    if rank == 0:
        torch.save(_adapter(m), out)
    torch.distributed.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("ds_cfg", [None, {"zero_optimization": {"stage": 2}, "gradient_clipping": 1.0,
                                           "train_micro_batch_size_per_gpu": "auto",
                                           "gradient_accumulation_steps": "auto"}])
def test_trainer_ddp_and_zero_world2_match_single(tmp_path, ds_cfg):
    out = str(tmp_path / "w2.pt")
    mp.spawn(_ddp_worker, args=(2, _port(), out, ds_cfg), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    # single process, per-device batch 2 = the two ranks' batch-1 shards of the same sample order
    ds = SyntheticLMDataset(512, 32, 8, seed=4)
    m = _model()
    single = Trainer(m, _args(tmp_path / "s", per_device_train_batch_size=2, save_steps=0, max_steps=3),
                     train_dataset=ds, data_collator=_PadCollator())
    single.train()
    want = _adapter(m)
    for k in want:
        assert torch.allclose(got[k], want[k], atol=2e-5), (k, (got[k] - want[k]).abs().max())


def test_trainer_zero3_saves_gathered_adapter(tmp_path):
    ds = SyntheticLMDataset(512, 32, 8, seed=5)
    m = _model()
    cfg = {"zero_optimization": {"stage": 3, "stage3_param_persistence_threshold": 0}}
    tr = Trainer(m, _args(tmp_path, max_steps=2, save_steps=2, deepspeed=cfg), train_dataset=ds,
                 data_collator=_PadCollator())
    tr.train()
    from safetensors.torch import load_file
    sd = load_file(str(tmp_path / "checkpoint-2" / "adapter_model.safetensors"))
    assert sd and all(v.numel() > 0 for v in sd.values())
    assert os.path.isdir(tmp_path / "checkpoint-2" / "global_step2")


def test_gemm4w_plan_policy():
    """gemm4w's host cost model (gemm4w.hip gemm4w_cfg; no device needed): tile shape and split-K per role of
    the Qwen3-8B step at M = 2048 — split only long reductions into an output that leaves CUs idle (gate|up dX,
    down fwd: 128 256x256 tiles -> 2 slices), the transposed-B 256x192 tile where it makes whole rounds."""
    from llm_in_practise_amd.ops._native import has_native, native
    if not has_native():
        pytest.skip("HIP extension not built")
    plan = lambda m, n, k, bt: tuple(native().gemm4w_plan_info(m, n, k, bt, False))  # noqa: E731  (splits, bn, bm)
    assert plan(2048, 4096, 24576, True) == (2, 256, 256)     # gate|up dX
    assert plan(2048, 4096, 12288, False) == (2, 256, 256)    # down fwd
    assert plan(2048, 4096, 6144, True)[0] == 1               # q|k|v dX: reduction not long enough to split
    assert plan(2048, 6144, 4096, False) == (1, 192, 256)     # q|k|v fwd: 8 x 32 = 256 tiles
    assert plan(2048, 12288, 4096, True) == (1, 192, 256)     # down dX: 512 tiles = 2 whole rounds
    assert plan(1024, 4096, 24576, True)[0] == 4              # 64 tiles -> 4 slices
