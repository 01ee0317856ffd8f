#!/usr/bin/env python3
"""Decode-shaped bf16 GEMM: gemm_skinny (HIP, split-K MFMA) vs hipBLASLt, Qwen3-8B shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) * 1000 / iters


C = native()
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288),
          "lm_head": (151936, 4096)}
tot = {}
for M in (1, 8, 16, 32, 64):
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        y = C.gemm_skinny(x, w, res)
        ref = x.float() @ w.float().t() + res.float()
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        assert err < 1e-2, (M, name, err)
        a = timeit(lambda: torch.addmm(res, x, w.t()))
        b = timeit(lambda: C.gemm_skinny(x, w, res))
        gb = N * K * 2 / 1e3
        tot[(M, "hipblaslt")] = tot.get((M, "hipblaslt"), 0) + (a if name != "lm_head" else 0)
        tot[(M, "skinny")] = tot.get((M, "skinny"), 0) + (b if name != "lm_head" else 0)
        print(f"M={M:3d} {name:8s} hipBLASLt {a:7.1f} us ({gb / a:5.0f} GB/s)  skinny {b:7.1f} us ({gb / b:5.0f} GB/s)"
              f"  err {err:.1e}", flush=True)
for k, v in sorted(tot.items()):
    print(f"TOTAL per layer M={k[0]:3d} {k[1]:10s} {v:7.1f} us")
