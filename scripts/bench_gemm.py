#!/usr/bin/env python3
"""Micro-benchmark of the NF4 / bf16 weight GEMMs at the Qwen3 shapes vs hipBLASLt bf16.

    python scripts/bench_gemm.py [--m 1024] [--iters 50]

Prints one line per (shape, direction) with µs and TFLOP/s; interleaves variants in one process.
"""
import argparse
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
    return ev[0].elapsed_time(ev[1]) * 1000 / iters  # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1024, 2048])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--model", default="8b")
    ap.add_argument("--impls", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--quick", action="store_true", help="NF4 impls + hipBLASLt only")
    a = ap.parse_args()
    C = native()
    h, f = (4096, 12288) if a.model == "8b" else (5120, 17408)
    shapes = {"qkv": (h + 2 * 1024, h), "o": (h, h), "gate_up": (2 * f, h), "down": (h, f)}
    torch.manual_seed(0)
    tot = {}
    for M in a.m:
        for name, (N, K) in shapes.items():
            w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
            q = quantize_nf4(w, 64, True)
            cf, cb, at = q.kernel_pack()
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            fl = 2 * M * N * K
            r = {}
            r["nf4_fwd_v2"] = timeit(lambda: C.gemm_nf4(x, cf, at, N, None, None, None), a.iters)
            r["nf4_bwd_v2"] = timeit(lambda: C.gemm_nf4_t(dy, cb, at, K, None, None), a.iters)
            r["bf16_fwd_gemm8"] = timeit(lambda: C.gemm8(x, w, None, None, None, 0), a.iters)
            if a.quick:
                r["bf16_fwd_hipblaslt"] = timeit(lambda: x @ w.t(), a.iters)
                r["bf16_bwd_hipblaslt"] = timeit(lambda: dy @ w, a.iters)
                for k, us in r.items():
                    tot[(M, k)] = tot.get((M, k), 0) + us
                    print(f"M={M:5d} {name:8s} N={N:6d} K={K:6d} {k:20s} {us:9.1f} us {fl / us / 1e6:8.1f} TF/s",
                          flush=True)
                continue
            r["bf16_fwd_hipblaslt"] = timeit(lambda: x @ w.t(), a.iters)
            r["bf16_bwd_hipblaslt"] = timeit(lambda: dy @ w, a.iters)
            r["bf16_fwd_lipa"] = timeit(lambda: C.gemm_bf16(x, w, None, None, None), a.iters)
            r["dequant+hipblaslt"] = timeit(lambda: x @ C.nf4_dequant(q.codes, None, q.qabsmax, q.absmax2, q.offset,
                                                                       _dq(), N, K).t(), a.iters)
            for k, us in r.items():
                tot[(M, k)] = tot.get((M, k), 0) + us
                print(f"M={M:5d} {name:8s} N={N:6d} K={K:6d} {k:20s} {us:9.1f} us {fl / us / 1e6:8.1f} TF/s",
                      flush=True)
    for (M, k), us in sorted(tot.items()):
        print(f"TOTAL M={M} {k:20s} {us:9.1f} us")


_DQ = None


def _dq():
    global _DQ
    if _DQ is None:
        from llm_in_practise_amd.quant.nf4 import dynamic_code
        _DQ = dynamic_code("cuda")
    return _DQ


if __name__ == "__main__":
    main()
