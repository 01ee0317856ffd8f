#!/usr/bin/env python3
"""Decode-shaped (small-M) GEMM micro-benchmark at the Qwen3-8B projection shapes:
the split-K bf16 skinny GEMM and the NF4 GEMV vs hipBLASLt (torch.matmul).  Reports µs and
effective weight-stream bandwidth (GB/s) — at M <= 64 these GEMMs are HBM-bound.

    python scripts/bench_skinny.py --m 1 8 16 32 64
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.nf4 import quantize_nf4  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1, 8, 16, 32, 64])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-nf4", action="store_true")
    a = ap.parse_args()
    C = native()
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288),
              "lm_head": (151936, 4096)}
    torch.manual_seed(0)
    for name, (N, K) in shapes.items():
        w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
        q = None if a.no_nf4 or name == "lm_head" else quantize_nf4(w, 64, True)
        for M in a.m:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            r = {"shape": name, "M": M, "N": N, "K": K}
            fns = {"hipblaslt_bf16": lambda: x @ w.t()}
            if hasattr(C, "gemm_skinny"):
                fns["skinny_bf16"] = lambda: C.gemm_skinny(x, w, None)
            if q is not None:
                sc = q.gemv_scales()
                if M <= 8:
                    fns["nf4_gemv"] = lambda: C.gemv_w4(x, q.codes, sc, None, N, 64, None)
            for k, fn in fns.items():
                us = timeit(fn, a.iters)
                wbytes = N * K * (0.5 if k.startswith("nf4") else 2)
                r[k + "_us"] = round(us, 1)
                r[k + "_GBs"] = round(wbytes / us / 1e3, 0)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
