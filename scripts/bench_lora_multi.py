"""The multi-adapter LoRA kernels in isolation at BASELINE #2's shapes (Qwen3-8B, M = 4096 tokens, rank 16,
dropout 0.05): q|k|v (3 adapters over x [M, 4096], dy column blocks 4096 / 1024 / 1024) and o (1 adapter).
Prints µs per call (min over interleaved rounds) and the compulsory HBM bytes / time.
    python scripts/bench_lora_multi.py [--pmc]   (--pmc: 8 plain repetitions for rocprofv3 --pmc)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

ext = native()
M, K, r, p = 4096, 4096, 16, 0.05
cols = [4096, 1024, 1024]
c0 = [0, 4096, 5120]
g = torch.Generator(device="cuda").manual_seed(0)
rnd = lambda *s: torch.randn(*s, device="cuda", generator=g).bfloat16()  # noqa: E731
x, xo = rnd(M, K), rnd(M, K)
dy, dyo = rnd(M, sum(cols)), rnd(M, K)
A3 = [rnd(r, K) * 0.05 for _ in cols]
bt3 = [rnd(r, n) * 0.05 for n in cols]
A1, bt1 = [rnd(r, K) * 0.05], [rnd(r, K) * 0.05]
masks3 = torch.empty(3, M, K // 8, dtype=torch.uint8, device="cuda")
masks1 = torch.empty(1, M, K // 8, dtype=torch.uint8, device="cuda")
xa32 = torch.zeros(M, 64, dtype=torch.bfloat16, device="cuda")
dB3 = [torch.zeros(n, r, device="cuda") for n in cols]
dA3 = [torch.zeros(r, K, device="cuda") for _ in cols]
dB1, dA1 = torch.zeros(K, r, device="cuda"), torch.zeros(r, K, device="cuda")


def fwd3():
    return ext.lora_proj_m(x, A3, [xa32[:, 16 * i:16 * i + 16] for i in range(3)], True, [p] * 3, [11, 12, 13],
                           [2.0] * 3, masks3)


def fwd1():
    return ext.lora_proj_m(xo, A1, [xa32[:, :16]], True, [p], [14], [2.0], masks1)


xa3, xa1 = fwd3(), fwd1()


def g3():
    return ext.lora_proj_cols(dy, c0, bt3, [2.0] * 3)


def g1():
    return ext.lora_proj_cols(dyo, [0], bt1, [2.0])


gl3, gl1 = g3(), g1()


def acc3():
    ext.lora_acc_jobs(list(xa3) + list(gl3), [dy] * 3 + [x] * 3, c0 + [0] * 3, cols + [K] * 3, dB3 + dA3,
                      [True] * 3 + [False] * 3, masks3, [-1] * 3 + [0, 1, 2], [0.0] * 3 + [p] * 3)


def acc1():
    ext.lora_acc_jobs([xa1[0], gl1[0]], [dyo, xo], [0, 0], [K, K], [dB1, dA1], [True, False], masks1, [-1, 0], [0.0, p])


def dxc3(rb=0):
    return ext.lora_dxc(list(gl3), A3, masks3, [p] * 3, rb)


MB = 1 << 20
cases = [  # name, fn, compulsory bytes
    ("proj_m q|k|v (x once, 3 keep planes)", fwd3, M * K * 2 + 3 * M * K // 8 + 3 * M * r * 6),
    ("proj_m o", fwd1, M * K * 2 + M * K // 8 + M * r * 6),
    ("proj_cols q|k|v (dy 6144 cols)", g3, M * sum(cols) * 2 + 3 * M * r * 4),
    ("proj_cols o", g1, M * K * 2 + M * r * 4),
    ("acc_jobs q|k|v (3 dB + 3 dA)", acc3, M * sum(cols) * 2 + 3 * M * K * 2 + 3 * M * K // 8),
    ("acc_jobs o (dB + dA)", acc1, 2 * M * K * 2 + M * K // 8),
    ("dxc q|k|v (C bf16 [M, K])", dxc3, M * K * 2 + 3 * M * K // 8 + 3 * M * r * 4),
] + [(f"dxc q|k|v rows/wave {16 * rb}", (lambda rb=rb: dxc3(rb)), M * K * 2 + 3 * M * K // 8 + 3 * M * r * 4)
     for rb in (1, 2, 4, 8)]


def timeit(fn, it=20):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1000


if "--pmc" in sys.argv:
    for _ in range(8):
        for _, fn, _ in cases:
            fn()
    torch.cuda.synchronize()
    sys.exit(0)
best = {n: 1e9 for n, _, _ in cases}
for _ in range(5):
    for n, fn, _ in cases:
        best[n] = min(best[n], timeit(fn))
for n, fn, b in cases:
    print(f"{n:42s} {best[n]:8.1f} us  {b / MB:7.1f} MB  {b / best[n] / 1e6:6.2f} TB/s", flush=True)
