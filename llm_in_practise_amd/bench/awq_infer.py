"""BASELINE config #5: QLoRA-tuned adapter merged into the base, then AWQ int4 W4A16 inference.

Reference flow: ``Fine-Tuning/deepseek-r1-0528-qwen3-8b-qlora-dist.py``
trains the adapter, ``merge_lora.py`` folds it into the bf16 base, LLM-Compressor AWQ quantises
the merged model (``Quantization/LLM-Compressor/AWQ/*``) and vLLM serves it; the quality bar is
``eval_qwen3_4b_awq.py:11-80`` (self-generated-token "PPL" proxy < 9.0).

Here, on random-init weights of the named architecture (no checkpoints are reachable):

1. build the bf16 model, attach a LoRA (r 8 / α 16 on q,v, non-zero B) and MERGE it;
2. time decode steps (hipGraph replay, ctx ``--ctx``) and a packed prefill on the bf16 model;
3. AWQ-quantise the merged model (activation-aware scale search on calibration tokens, then
   group-128 asymmetric int4) — or RTN with ``--method rtn``;
4. measure the same steps on the W4A16 model (``gemv_w4`` at M ≤ 2, ``w4mm`` to 32 rows, gemm4w W4=2 above),
   plus the quality of int4 against bf16: next-token KL, top-1 agreement and the self-PPL proxy
   of both (random weights: the absolute PPL is not comparable to the reference's 8.19 / 9.0 bar,
   so the int4 / bf16 ratio is what is reported — "parity unpinned");
5. optionally serve ``--serve-requests`` requests through the ServingEngine (continuous batching)
   and report output tok/s.

    python -m llm_in_practise_amd.bench.awq_infer --model qwen3-8b --method awq --out awq.json
"""
from __future__ import annotations

import argparse
import json
import math
import time

import torch


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _merged_model(name: str, r: int, alpha: int, seed: int, device):
    from ..models.qwen3 import Qwen3ForCausalLM, qwen3_config
    from ..peft.lora import LoraConfig, get_peft_model
    torch.manual_seed(seed)
    base = Qwen3ForCausalLM.from_config(qwen3_config(name), dtype=torch.bfloat16, device=device)
    peft = get_peft_model(base, LoraConfig(r=r, lora_alpha=alpha, target_modules=["q_proj", "v_proj"],
                                           lora_dropout=0.0))
    with torch.no_grad():                          # a "trained" adapter: B ≠ 0
        for n, p in peft.named_parameters():
            if "lora_B" in n:
                p.normal_(0.0, 0.02)
    m = peft.merge_and_unload()
    m.requires_grad_(False)
    return m.eval()


@torch.no_grad()
def _decode_steps(lm, batches, ctx, steps, max_len):
    from ..infer.graphs import DecodeGraphs
    from ..models.common import KVCache
    cfg = lm.config
    dev = next(lm.parameters()).device
    B = max(batches)
    cache = KVCache(cfg.num_hidden_layers, B, max_len, cfg.num_key_value_heads, cfg.head_dim, torch.bfloat16, dev)
    cache.pos = torch.full((B,), ctx, dtype=torch.long, device=dev)
    tok = torch.randint(0, cfg.vocab_size, (B,), device=dev)
    if dev.type == "cuda":                         # hipGraph replay, as the serving engine decodes
        dg = DecodeGraphs(lm, cache, B, buckets=sorted(set(batches)))
        step = dg.step
    else:
        dg = None

        def step(t, n):
            return lm.model(t[:, None], None, cache.head_rows(n), None) @ lm.lm_head.weight.t()
    rows = []
    for n in batches:
        for _ in range(3):
            step(tok[:n], n)
        cache.pos.fill_(ctx)
        _sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(tok[:n], n)
            cache.pos.fill_(ctx)
        _sync()
        ms = (time.perf_counter() - t0) / steps * 1e3
        rows.append({"batch": n, "ctx": ctx, "step_ms": round(ms, 3), "tok_per_s": round(n / ms * 1e3, 1)})
    del dg, cache
    torch.cuda.empty_cache() if torch.cuda.is_available() else None
    return rows


@torch.no_grad()
def _prefill(lm, B, S, steps):
    dev = next(lm.parameters()).device
    ids = torch.randint(0, lm.config.vocab_size, (B, S), device=dev)
    for _ in range(2):
        lm.model(ids, None, None, None)
    _sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        lm.model(ids, None, None, None)
    _sync()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"batch": B, "seq": S, "ms": round(ms, 3), "tok_per_s": round(B * S / ms * 1e3, 1)}


@torch.no_grad()
def _next_token_logp(lm, ids):
    return torch.log_softmax(lm(ids).logits.float(), -1)


def _serve(lm, n_req, max_tokens, max_batch):
    from ..infer.engine import SamplingParams, ServingEngine
    from ..train.data import ByteTokenizer
    eng = ServingEngine(lm, ByteTokenizer(), model_name="awq-int4", max_batch=max_batch, max_model_len=1024)
    try:
        params = SamplingParams(max_tokens=max_tokens, temperature=0.0, ignore_eos=True)
        eng.complete("warm up " * 8, SamplingParams(max_tokens=4, temperature=0.0))
        prompts = [f"request {i}: " + "tell me about MI355X " * 6 for i in range(n_req)]
        t0 = time.perf_counter()
        outs = [eng.submit(p, params) for p in prompts]
        toks = 0
        for q in outs:
            while True:
                kind, val = q.out.get(timeout=600)
                if kind == "final":
                    toks += val["completion_tokens"]
                    break
                if kind == "error":
                    raise RuntimeError(val)
        dt = time.perf_counter() - t0
        return {"requests": n_req, "max_tokens": max_tokens, "duration_s": round(dt, 3),
                "output_tok_per_s": round(toks / dt, 1)}
    finally:
        eng.shutdown()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model", default="qwen3-8b")
    ap.add_argument("--method", default="awq", choices=["awq", "rtn"])
    ap.add_argument("--group-size", type=int, default=128)
    ap.add_argument("--lora-r", type=int, default=8)
    ap.add_argument("--lora-alpha", type=int, default=16)
    ap.add_argument("--calib", type=int, default=8, help="calibration sequences (AWQ)")
    ap.add_argument("--calib-len", type=int, default=256)
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 64, 256])
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--max-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--prefill", type=int, nargs=2, default=[4, 512], metavar=("B", "S"))
    ap.add_argument("--ppl-prompts", type=int, default=4)
    ap.add_argument("--ppl-new", type=int, default=64)
    ap.add_argument("--serve-requests", type=int, default=0)
    ap.add_argument("--serve-tokens", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    from ..quant.eval import self_ppl
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    lm = _merged_model(a.model, a.lora_r, a.lora_alpha, a.seed, dev)
    res: dict = {"config": {"model": a.model, "method": a.method, "group_size": a.group_size,
                            "merged_lora": {"r": a.lora_r, "alpha": a.lora_alpha, "targets": ["q_proj", "v_proj"]},
                            "data": "synthetic random-init weights and tokens"}}
    g = torch.Generator().manual_seed(a.seed + 1)
    V = lm.config.vocab_size
    eval_ids = torch.randint(0, V, (4, 128), generator=g).to(dev)
    prompts = [torch.randint(0, V, (32,), generator=g).to(dev) for _ in range(a.ppl_prompts)]
    calib = [torch.randint(0, V, (1, a.calib_len), generator=g) for _ in range(a.calib)]

    lm.fuse_projections()
    res["bf16"] = {"decode": _decode_steps(lm, a.batches, a.ctx, a.steps, a.max_len),
                   "prefill": _prefill(lm, *a.prefill, a.steps // 2 or 1),
                   "self_ppl": self_ppl(lm, prompts, a.ppl_new),
                   "weight_bytes": sum(p.numel() * p.element_size() for n, p in lm.named_parameters()
                                       if n.startswith("model.layers") and p.dim() == 2)}
    ref_logp = _next_token_logp(lm, eval_ids)
    lm.invalidate_fusion()

    t0 = time.perf_counter()
    if a.method == "awq":
        from ..quant.awq import awq_quantize_model
        awq_quantize_model(lm, calib, a.group_size)
    else:
        from ..quant.gptq import replace_with_int4
        from ..quant.int4 import quantize_rtn
        ws = {n: quantize_rtn(mod.weight.detach(), a.group_size) for n, mod in lm.named_modules()
              if isinstance(mod, torch.nn.Linear) and n.startswith("model.layers")}
        replace_with_int4(lm, ws)
    _sync()
    res["quantize_s"] = round(time.perf_counter() - t0, 2)
    torch.cuda.empty_cache() if torch.cuda.is_available() else None
    lm.fuse_projections()
    from ..quant.int4 import Int4Linear
    int4_bytes = sum(m.int4.nbytes() for m in lm.modules() if isinstance(m, Int4Linear))
    logp = _next_token_logp(lm, eval_ids)
    kl = (ref_logp.exp() * (ref_logp - logp)).sum(-1).mean().item()
    agree = (ref_logp.argmax(-1) == logp.argmax(-1)).float().mean().item()
    res["int4"] = {"decode": _decode_steps(lm, a.batches, a.ctx, a.steps, a.max_len),
                   "prefill": _prefill(lm, *a.prefill, a.steps // 2 or 1),
                   "self_ppl": self_ppl(lm, prompts, a.ppl_new),
                   "weight_bytes": int4_bytes, "kl_vs_bf16": kl, "top1_agree_vs_bf16": agree}
    res["int4"]["self_ppl_ratio_vs_bf16"] = res["int4"]["self_ppl"] / res["bf16"]["self_ppl"]
    res["decode_speedup"] = {str(b["batch"]): round(b["step_ms"] / q["step_ms"], 3)
                             for b, q in zip(res["bf16"]["decode"], res["int4"]["decode"])}
    if a.serve_requests:
        res["int4"]["serve"] = _serve(lm, a.serve_requests, a.serve_tokens, max(a.batches))
    for k in ("bf16", "int4"):
        if not math.isfinite(res[k]["self_ppl"]):
            res[k]["self_ppl"] = None
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return res


if __name__ == "__main__":
    main()
