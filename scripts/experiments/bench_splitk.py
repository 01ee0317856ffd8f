#!/usr/bin/env python3
"""gate_up / LM-head backward dX = dY·W at M=2048: plain hipBLASLt vs batched split-K (bmm + sum)."""
import torch

def timeit(fn, iters=30):
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

M = 2048
for name, (N, K) in {"gate_up": (24576, 4096), "down": (4096, 12288), "qkv": (6144, 4096)}.items():
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * N * K
    ref = dy.float() @ w.float()
    row = [f"{name:8s} plain {timeit(lambda: dy @ w):7.1f} us"]
    for s in (2, 3, 4, 6, 8):
        if N % s:
            continue
        def f():
            return torch.bmm(dy.view(M, s, N // s).transpose(0, 1), w.view(s, N // s, K)).sum(0, dtype=torch.float32).to(torch.bfloat16)
        def g():
            return torch.bmm(dy.view(M, s, N // s).transpose(0, 1), w.view(s, N // s, K)).sum(0)
        err = ((f().float() - ref).abs().max() / ref.abs().max()).item()
        row.append(f"split{s} fp32sum {timeit(f):7.1f} bf16sum {timeit(g):7.1f} (err {err:.1e})")
    print("  ".join(row), flush=True)
