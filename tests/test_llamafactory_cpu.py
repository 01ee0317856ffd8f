"""``lipa lf train|export <yaml>`` — the LLaMA-Factory recipe path on CPU."""
import json
import os

import torch

from llm_in_practise_amd.cli.llamafactory import load_lf_yaml, resolve_datasets
from llm_in_practise_amd.cli.main import main

# same shape as the reference recipe, including its malformed ``dataset:`` scalar + list items
RECIPE = """### model
model_name_or_path: random:qwen3-tiny  # comment
template: deepseekr1

### method
stage: sft
do_train: true
finetuning_type: lora
lora_target: all

### dataset
dataset: my_identity
  - demo_alpaca
cutoff_len: 64
overwrite_cache: true

### output
output_dir: {out}
logging_steps: 1
save_steps: 1000

### train
per_device_train_batch_size: 2
gradient_accumulation_steps: 2
learning_rate: 1.0e-3
num_train_epochs: 1.0
max_steps: 3
lr_scheduler_type: cosine
dataset_dir: {data}
"""


def _write(tmp_path):
    data = tmp_path / "data"
    data.mkdir()
    (data / "demo_alpaca.json").write_text(json.dumps(
        [{"instruction": f"q{i}", "input": "ctx" if i % 2 else "", "output": f"a{i}"} for i in range(6)]))
    (data / "ident.jsonl").write_text("\n".join(json.dumps({"query": "who?", "response": "I am {{NAME}}"})
                                                for _ in range(4)))
    (data / "dataset_info.json").write_text(json.dumps({"my_identity": {"file_name": "ident.jsonl"}}))
    cfg = tmp_path / "sft.yaml"
    cfg.write_text(RECIPE.format(out=tmp_path / "out", data=data))
    return cfg, data


def test_malformed_recipe_loads_as_list(tmp_path):
    cfg, data = _write(tmp_path)
    d = load_lf_yaml(str(cfg))
    assert d["dataset"] == ["my_identity", "demo_alpaca"] and d["learning_rate"] == 1e-3
    recs = resolve_datasets(d["dataset"], str(data))
    assert len(recs) == 10 and recs[5]["query"] == "q1\nctx"


def test_lf_train_then_export(tmp_path):
    cfg, _ = _write(tmp_path)
    main(["lf", "train", str(cfg), "--tokenizer", "bytes"])
    out = tmp_path / "out"
    assert (out / "adapter_model.safetensors").exists()
    ac = json.loads((out / "adapter_config.json").read_text())
    assert ac["r"] == 8 and ac["lora_alpha"] == 16
    exp = tmp_path / "merged"
    main(["lf", "export", str(cfg), f"adapter_name_or_path={out}", f"export_dir={exp}"])
    assert (exp / "model.safetensors").exists() and (exp / "config.json").exists()
