#!/usr/bin/env python3
"""NF4 → bf16 dequant kernel variants at the Qwen3-8B layer shapes (GB/s of HBM traffic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.nf4 import quantize_nf4  # noqa: E402


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
for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288)}.items():
    q = quantize_nf4((0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16), 64, True)
    sc = q.gemv_scales()
    nbytes = N * K * 2 + N * K // 2 + sc.numel() * 4
    row = [f"{name:8s}"]
    ref = None
    for v in (2, 3):
        C.set_dequant_variant(v)
        out = C.nf4_dequant_fast(q.codes, sc, N, K)
        ref = out if ref is None else ref
        assert torch.equal(out, ref)
        us = timeit(lambda: C.nf4_dequant_fast(q.codes, sc, N, K))
        row.append(f"v{v} {us:7.1f} us {nbytes / us / 1e3:6.0f} GB/s")
    c2 = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    us = timeit(lambda: c2.copy_(ref))
    row.append(f"| bf16 copy {us:7.1f} us {2 * N * K * 2 / us / 1e3:6.0f} GB/s")
    print("  ".join(row), flush=True)
C.set_dequant_variant(3)
