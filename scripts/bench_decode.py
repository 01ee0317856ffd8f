#!/usr/bin/env python3
"""Decode-step microbenchmark: eager vs hipGraph replay, per batch size (random-init weights).

    python scripts/bench_decode.py --model qwen3-8b --batches 1 8 32 64 --ctx 1024
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_in_practise_amd.infer.graphs import DecodeGraphs  # noqa: E402
from llm_in_practise_amd.models.common import KVCache  # noqa: E402
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config  # noqa: E402
from llm_in_practise_amd.peft.lora import quantize_model_nf4  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-8b")
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 32, 64])
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--max-len", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--nf4", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    lm = Qwen3ForCausalLM.from_config(qwen3_config(a.model), dtype=torch.bfloat16, device=dev).eval()
    lm.requires_grad_(False)
    if a.nf4:
        quantize_model_nf4(lm)
    lm.fuse_projections()
    cfg = lm.config
    B = max(a.batches)
    cache = KVCache(cfg.num_hidden_layers, B, a.max_len, cfg.num_key_value_heads, cfg.head_dim, torch.bfloat16, dev)
    cache.pos = torch.full((B,), a.ctx, dtype=torch.long, device=dev)
    tok = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    rows = []
    with torch.no_grad():
        for n in a.batches:
            view = cache.head_rows(n)

            def eager():
                h = lm.model(tok[:n, None], None, view, None)
                return h @ lm.lm_head.weight.t()
            for _ in range(3):
                eager()
            cache.pos.fill_(a.ctx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eager()
                cache.pos.fill_(a.ctx)
            torch.cuda.synchronize()
            t_eager = (time.perf_counter() - t0) / a.steps * 1e3
            rows.append({"batch": n, "ctx": a.ctx, "eager_ms": round(t_eager, 3)})
        if not a.no_graph:
            cache.pos.fill_(a.ctx)
            t0 = time.perf_counter()
            dg = DecodeGraphs(lm, cache, B, buckets=sorted(set(a.batches)))
            t_cap = time.perf_counter() - t0
            for r in rows:
                n = r["batch"]
                for _ in range(3):
                    dg.step(tok[:n], n)
                cache.pos.fill_(a.ctx)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    dg.step(tok[:n], n)
                    cache.pos.fill_(a.ctx)
                torch.cuda.synchronize()
                r["graph_ms"] = round((time.perf_counter() - t0) / a.steps * 1e3, 3)
                r["graph_tok_per_s"] = round(n / r["graph_ms"] * 1e3, 1)
                r["capture_s"] = round(t_cap, 2)
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
