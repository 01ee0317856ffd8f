"""torch.profiler view of one bench step: which aten ops launch the non-HIP-kernel work
(copies, adds, fills) and from which Python frames.  python scripts/torch_prof_step.py"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config  # noqa: E402
from llm_in_practise_amd.optim.adamw import build_optimizer  # noqa: E402
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4  # noqa: E402

dev = torch.device("cuda", 0)
cfg = qwen3_config(sys.argv[1] if len(sys.argv) > 1 else "qwen3-8b")
model = Qwen3ForCausalLM.from_config(cfg, dtype=torch.bfloat16, device=dev, seed=1)
quantize_model_nf4(model)
pm = get_peft_model(model, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.1, target_modules=["q_proj", "v_proj"]))
model.fuse_projections()
pm.train()
opt = build_optimizer("paged_adamw_8bit", [p for p in pm.parameters() if p.requires_grad], 5e-5, max_grad_norm=1.0)
ids = torch.randint(0, cfg.vocab_size, (4, 512), device=dev)


def step():
    out = pm(ids, labels=ids, num_micro_batches=2)
    out.loss.backward()
    opt.clip_grad_norm_(1.0)
    opt.step()
    opt.zero_grad()


for _ in range(2):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=50,
                                                        max_shapes_column_width=60))
for ev in sorted(prof.key_averages(group_by_stack_n=8), key=lambda e: -e.device_time_total):
    if ev.key.startswith("aten::") and ev.device_time_total > 0 and ev.key not in ("aten::mm", "aten::matmul"):
        print(f"{ev.key:30s} calls={ev.count:5d} cuda={ev.device_time_total / 1000:8.3f} ms")
        for fr in ev.stack[:8]:
            print("      ", fr)
