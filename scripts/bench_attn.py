"""Attention microbenchmark: our HIP flash attention fwd/bwd vs torch SDPA at the bench shapes.

    python scripts/bench_attn.py [--B 4 --S 512 --hq 32 --hkv 8 --d 128]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--no-sdpa", action="store_true", help="skip the torch SDPA comparison")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    B, S, hq, hkv, d = a.B, a.S, a.hq, a.hkv, a.d
    ext = native()
    T = B * S
    q = torch.randn(T, hq * d, device="cuda").to(torch.bfloat16)
    kv = torch.randn(T, 2 * hkv * d, device="cuda").to(torch.bfloat16)
    k, v = kv[:, :hkv * d], kv[:, hkv * d:]
    scale = 1 / math.sqrt(d)
    o, lse = ext.attn_fwd(q, k, v, None, B, S, hq, hkv, d, True, scale)
    do = torch.randn_like(o)
    t_f = timeit(lambda: ext.attn_fwd(q, k, v, None, B, S, hq, hkv, d, True, scale), a.iters)
    t_b = timeit(lambda: ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, d, True, scale, 0.0, 0), a.iters)
    fl = 4 * B * hq * S * S * d / 2  # causal fwd
    if a.no_sdpa:
        print(json.dumps({"shape": [B, S, hq, hkv, d], "ours_fwd_us": round(t_f, 1), "ours_bwd_us": round(t_b, 1),
                          "ours_fwd_TFs": round(fl / t_f / 1e6, 1), "ours_bwd_TFs": round(2.5 * fl / t_b / 1e6, 1)}))
        return
    qs = q.view(B, S, hq, d).transpose(1, 2)
    ks = k.reshape(B, S, hkv, d).transpose(1, 2).repeat_interleave(hq // hkv, 1).contiguous()
    vs = v.reshape(B, S, hkv, d).transpose(1, 2).repeat_interleave(hq // hkv, 1).contiguous()
    sd = lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=True)
    t_sf = timeit(sd)
    qg, kg, vg = (t.detach().requires_grad_(True) for t in (qs, ks, vs))
    og = torch.nn.functional.scaled_dot_product_attention(qg, kg, vg, is_causal=True)
    gd = torch.randn_like(og)
    t_sb = timeit(lambda: torch.autograd.grad(og, (qg, kg, vg), gd, retain_graph=True))
    print(json.dumps({"shape": [B, S, hq, hkv, d], "ours_fwd_us": round(t_f, 1), "ours_bwd_us": round(t_b, 1),
                      "ours_fwd_TFs": round(fl / t_f / 1e6, 1), "ours_bwd_TFs": round(2.5 * fl / t_b / 1e6, 1),
                      "sdpa_fwd_us": round(t_sf, 1), "sdpa_bwd_us": round(t_sb, 1)}))


if __name__ == "__main__":
    main()
