"""Cost of the LoRA terms inside gemm4w (the prologue K-step of the q|k|v forward, the masked dX term of the
q|k|v dX) against the plain gemm4w on the same shape / tile — Qwen3-8B q|k|v, q_proj + v_proj adapters r 8.
    python scripts/bench_lora_gemm.py [M ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

ext = native()


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        st.record()
        for _ in range(it):
            fn()
        en.record()
        torch.cuda.synchronize()
        best = min(best, st.elapsed_time(en) / it * 1000)
    return best


rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
for M in [int(m) for m in (sys.argv[1:] or [1024, 2048])]:
    N, K, r = 6144, 4096, 8
    x, w = rnd(M, K), rnd(N, K) * 0.02
    xa = rnd(M, 32)
    bq, bv = rnd(4096, r) * 0.1, rnd(1024, r) * 0.1
    fwd_plain = timeit(lambda: ext.gemm4w(x, w, None, 1, False))
    fwd_lora = timeit(lambda: ext.gemm4w_lora(x, w, None, 0, None, xa, [bq, bv], [0, 5120], [0, 8], [None, None]))
    dy = rnd(M, N)
    g = [torch.randn(M, r, device="cuda"), torch.randn(M, r, device="cuda")]
    a = [rnd(r, K) * 0.1, rnd(r, K) * 0.1]
    masks = torch.randint(0, 256, (2, M, K // 8), device="cuda", dtype=torch.uint8)
    dx_plain = timeit(lambda: ext.gemm4w(dy, w, None, 1, True))
    dx_lora = timeit(lambda: ext.gemm4w_loradx(dy, w, None, 0, g, a, masks, [0.1, 0.1], 0, 0))
    print(f"M={M}: q|k|v fwd plain {fwd_plain:6.1f} us  +LoRA prologue {fwd_lora:6.1f} us | "
          f"dX plain {dx_plain:6.1f} us  +LoRA dX term {dx_lora:6.1f} us", flush=True)
