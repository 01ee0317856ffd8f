#!/usr/bin/env python3
"""hipBLASLt dX = dY·W with W [N,K] row-major (as dequantised) vs a transposed copy Wt [K,N]."""
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
for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288)}.items():
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    wt = w.t().contiguous()
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * N * K
    a = timeit(lambda: dy @ w)
    b = timeit(lambda: dy @ wt.t())
    c = timeit(lambda: x @ w.t())
    t = timeit(lambda: w.t().contiguous())
    print(f"{name:8s} bwd dy@W {a:7.1f} us ({fl/a/1e6:6.0f} TF/s)  bwd dy@Wt.T {b:7.1f} us ({fl/b/1e6:6.0f} TF/s)  "
          f"fwd {c:7.1f} us  transpose-copy {t:6.1f} us", flush=True)
