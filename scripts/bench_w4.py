#!/usr/bin/env python3
"""W4A16 decode-batch GEMM microbenchmark (Qwen3-8B projection shapes): bf16 hipBLASLt vs the
int4 kernels — gemv_w4 (M <= 8), gemm_int4 (MFMA tile kernel), gemm_w4_skinny (split-K weight
streaming).  Prints one JSON line per (shape, M)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.int4 import quantize_rtn  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def main():
    nat = native()
    Ms = [int(m) for m in (sys.argv[1:] or [1, 2, 8, 16, 32, 64, 128, 256])]
    for name, (N, K) in SHAPES.items():
        w = torch.randn(N, K, device="cuda") * 0.02
        wb = w.to(torch.bfloat16)
        q = quantize_rtn(w, 128)
        sc, bi = q.gemv_tables()
        cf, st, bt = q.kernel_pack()
        ref_w = q.dequantize()
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            ref = x.float() @ ref_w.t()
            row = {"shape": name, "M": M, "N": N, "K": K}
            row["bf16_us"] = round(timeit(lambda: x @ wb.t()), 2)
            if M <= 8:
                row["gemv_w4_us"] = round(timeit(lambda: nat.gemv_w4(x, q.codes, sc, bi, N, 128, None)), 2)
            row["gemm_int4_us"] = round(timeit(lambda: nat.gemm_int4(x, cf, st, bt, N, None, None, None)), 2)
            if M <= 64:
                row["w4_skinny_us"] = round(timeit(lambda: nat.gemm_w4_skinny(x, q.codes, sc, bi, N, 128, None)), 2)
                y = nat.gemm_w4_skinny(x, q.codes, sc, bi, N, 128, None)
                row["w4_skinny_relerr"] = float(((y.float() - ref).norm() / ref.norm()).item())
                row["w4_skinny_GBs"] = round(N * K / 2 / (row["w4_skinny_us"] * 1e-6) / 1e9, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
