"""Host-side cost of one bench step, phase by phase: the time Python takes to ENQUEUE the forward,
the backward and the optimizer (the GPU is drained before each phase, so no phase waits on the
device), against the GPU time of the same phases.  python scripts/host_overhead.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config  # noqa: E402
from llm_in_practise_amd.optim.adamw import build_optimizer  # noqa: E402
from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model, quantize_model_nf4  # noqa: E402

dev = torch.device("cuda", 0)
cfg = qwen3_config(sys.argv[1] if len(sys.argv) > 1 else "qwen3-8b")
model = Qwen3ForCausalLM.from_config(cfg, dtype=torch.bfloat16, device=dev, seed=1)
quantize_model_nf4(model)
pm = get_peft_model(model, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.05, target_modules=["q_proj", "v_proj"]))
model.fuse_projections()
pm.train()
opt = build_optimizer("paged_adamw_8bit", [p for p in pm.parameters() if p.requires_grad], 5e-5, max_grad_norm=1.0)
ids = torch.randint(0, cfg.vocab_size, (4, 512), device=dev)


def phases():
    t = [time.perf_counter()]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    out = pm(ids, labels=ids, num_micro_batches=2)
    t.append(time.perf_counter())
    e[1].record()
    out.loss.backward()
    t.append(time.perf_counter())
    e[2].record()
    opt.clip_grad_norm_(1.0)
    opt.step()
    opt.zero_grad()
    t.append(time.perf_counter())
    e[3].record()
    torch.cuda.synchronize()
    host = [1e3 * (t[i + 1] - t[i]) for i in range(3)]
    gpu = [e[i].elapsed_time(e[i + 1]) for i in range(3)]
    del out
    return host, gpu


for _ in range(3):
    phases()
for _ in range(3):
    h, g = phases()
    print(f"host enqueue ms: fwd {h[0]:6.2f} bwd {h[1]:6.2f} opt {h[2]:6.2f} | gpu ms: fwd {g[0]:6.2f} "
          f"bwd {g[1]:6.2f} opt {g[2]:6.2f}", flush=True)
