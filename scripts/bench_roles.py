"""Every frozen-base GEMM role of the Qwen3-8B QLoRA step (M = 2048 tokens, bf16 expansion as B) in its two
forms: the hand-written gemm4w launch the step ships (epilogues fused) vs hipBLASLt (lt_linear / lt_dx, the
library path of LIPA_GEMM=lt) + the separate elementwise pass it needs.  Interleaved rounds, min per form.
    python scripts/bench_roles.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

ext = native()
M, d, f = 2048, 4096, 12288
rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
w_qkv, w_o, w_gu, w_d = rnd(6144, d) * 0.02, rnd(d, d) * 0.02, rnd(2 * f, d) * 0.02, rnd(d, f) * 0.02
x, h, res = rnd(M, d), rnd(M, f), rnd(M, d)
dy_qkv, dy_d, dy_gu = rnd(M, 6144), rnd(M, d), rnd(M, 2 * f)
gu = rnd(M, 2 * f)

roles = {
    "qkv fwd": (lambda: ext.gemm4w(x, w_qkv, None, 0, False), lambda: ext.lt_linear(x, w_qkv, None, True)),
    "qkv dX": (lambda: ext.gemm4w(dy_qkv, w_qkv, None, 0, True), lambda: ext.lt_dx(dy_qkv, w_qkv, 1, True, None)),
    "o fwd + res": (lambda: ext.gemm4w(x, w_o, res, 0, False), lambda: ext.lt_linear(x, w_o, res, True)),
    "o dX": (lambda: ext.gemm4w(dy_d, w_o, None, 0, True), lambda: ext.lt_dx(dy_d, w_o, 1, True, None)),
    "gate|up fwd + SwiGLU": (lambda: ext.gemm4w_swiglu(x, w_gu, None, f),
                             lambda: ext.swiglu_fwd(ext.lt_linear(x, w_gu, None, True))),
    "down fwd + res": (lambda: ext.gemm4w(h, w_d, res, 0, False), lambda: ext.lt_linear(h, w_d, res, True)),
    "down dX + dSwiGLU": (lambda: ext.gemm4w_dswiglu(dy_d, w_d, gu, None),
                          lambda: ext.swiglu_bwd(ext.lt_dx(dy_d, w_d, 1, True, None), gu)),
    "gate|up dX": (lambda: ext.gemm4w(dy_gu, w_gu, None, 0, True), lambda: ext.lt_dx(dy_gu, w_gu, 2, True, None)),
}


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1000


best = {k: [1e9, 1e9] for k in roles}
for _ in range(4):
    for k, (a, b) in roles.items():
        best[k][0] = min(best[k][0], timeit(a))
        best[k][1] = min(best[k][1], timeit(b))
tot = [0.0, 0.0]
for k, (g, lt) in best.items():
    tot[0] += g
    tot[1] += lt
    print(f"{k:24s} gemm4w {g:7.1f} us   hipBLASLt(+pass) {lt:7.1f} us   {'gemm4w' if g <= lt else 'library'}", flush=True)
print(f"{'per layer':24s} gemm4w {tot[0]:7.1f} us   hipBLASLt(+pass) {tot[1]:7.1f} us   best-of {sum(min(v) for v in best.values()):7.1f} us")
