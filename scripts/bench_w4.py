#!/usr/bin/env python3
"""W4A16 decode-batch GEMM microbenchmark (Qwen3-8B projection shapes): bf16 (hipBLASLt, gemm4w) vs the
int4 kernels — gemv_w4 (M <= 8), w4mm (M <= 64, byte-permute dequant + MFMA, per-K-slice-count columns),
w4g (M <= 256, the same dequant tiled for decode batches, per-K-slice-count columns), gemm4w W4=2 (affine table expanded in-kernel).  Prints one JSON line per (shape, M)."""
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
        sc2 = q.w4mm_table()
        gc, gst, gzt = q.g4w_pack()
        ref_w = q.dequantize()
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            ref = x.float() @ ref_w.t()
            row = {"shape": name, "M": M, "N": N, "K": K}
            row["bf16_us"] = round(timeit(lambda: x @ wb.t()), 2)
            if M >= 16:
                row["bf16_g4w_us"] = round(timeit(lambda: nat.gemm4w(x, wb, None, 0, False)), 2)
            if nat.w4mm_ok(M, N, K, 128):
                row["w4mm_us"] = round(timeit(lambda: nat.w4mm(x, q.codes, sc2, N, 128, None, 0)), 2)
                y = nat.w4mm(x, q.codes, sc2, N, 128, None, 0)
                row["w4mm_relerr"] = float(((y.float() - ref).norm() / ref.norm()).item())
                row["w4mm_GBs"] = round(N * K / 2 / (row["w4mm_us"] * 1e-6) / 1e9, 1)
                for nkb in (1, 2, 4, 8):
                    if (K // 128) % nkb == 0:
                        row[f"w4mm_nkb{nkb}_us"] = round(timeit(lambda: nat.w4mm(x, q.codes, sc2, N, 128, None, nkb)), 2)
            if nat.w4g_ok(M, N, K, 128):
                row["w4g_us"] = round(timeit(lambda: nat.w4g(x, q.codes, sc2, N, 128, None, 0)), 2)
                y = nat.w4g(x, q.codes, sc2, N, 128, None, 0)
                row["w4g_relerr"] = float(((y.float() - ref).norm() / ref.norm()).item())
                row["w4g_ks"] = nat.w4g_splits(M, N, K)
                for ks in (1, 2, 4, 8):
                    if (K // 128) % ks == 0 and ks != row["w4g_ks"]:
                        row[f"w4g_ks{ks}_us"] = round(timeit(lambda: nat.w4g(x, q.codes, sc2, N, 128, None, ks)), 2)
            if M > 8:
                row["g4w_int4_us"] = round(timeit(lambda: nat.gemm4w(x, gc, None, 0, False, 0, 0, gst, N, gzt)), 2)
            if M >= 128:   # the prefill form: one bf16 expansion + the bf16 gemm4w
                row["expand_us"] = round(timeit(lambda: nat.int4_dequant(q.codes, sc, bi, N, K, 128)), 2)
                row["expand_g4w_us"] = round(timeit(lambda: nat.gemm4w(x, nat.int4_dequant(q.codes, sc, bi, N, K, 128),
                                                                    None, 0, False)), 2)
                y = nat.gemm4w(x, nat.int4_dequant(q.codes, sc, bi, N, K, 128), None, 0, False)
                row["expand_relerr"] = float(((y.float() - ref).norm() / ref.norm()).item())
            if M <= 8:
                row["gemv_w4_us"] = round(timeit(lambda: nat.gemv_w4(x, q.codes, sc, bi, N, 128, None)), 2)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
