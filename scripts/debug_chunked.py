"""Debug: whole-prompt prefill vs chunked prefill hidden states (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.models.common import KVCache  # noqa: E402
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config  # noqa: E402
import llm_in_practise_amd.ops.attention as A  # noqa: E402

torch.manual_seed(0)
cfg = qwen3_config("qwen3-small", vocab_size=256)
m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.bfloat16, device="cuda")
m.eval()
L = 200
ids = torch.randint(0, 256, (1, L), device="cuda")
hd = cfg.head_dim if hasattr(cfg, "head_dim") else cfg.hidden_size // cfg.num_attention_heads
with torch.no_grad():
    c1 = KVCache(cfg.num_hidden_layers, 1, 512, cfg.num_key_value_heads, hd, torch.bfloat16, "cuda")
    h1 = m.model(ids, None, c1, None)
    for chunk in (64, 50):
        c2 = KVCache(cfg.num_hidden_layers, 1, 512, cfg.num_key_value_heads, hd, torch.bfloat16, "cuda")
        hs = []
        for s in range(0, L, chunk):
            c2.len = s
            hs.append(m.model(ids[:, s:s + chunk], None, c2, None))
        h2 = torch.cat(hs)
        err = ((h2.float() - h1.float()).norm(dim=-1) / h1.float().norm(dim=-1))
        print("chunk", chunk, "max row relerr", err.max().item(), "first bad row", (err > 0.05).nonzero()[:3].flatten().tolist())
        kd = (c2.k[0][0, :L].float() - c1.k[0][0, :L].float()).abs().max().item()
        print("  layer0 K cache max diff", kd)
