"""Per-round fixed cost of gemm4w: time the same grid at several K (M = 2048, the gate|up fwd + SwiGLU epilogue,
the plain NT 256x256 and the transposed-B 256x192 down-dX + dSwiGLU) and fit t = a + b·K-tiles.  The intercept
a is the prologue + epilogue + launch cost every round of tiles pays (what a persistent tile loop could hide)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, it=10):
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


ext = native()
rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
M, F = 2048, 12288
for name in ("swiglu_fwd", "nt256", "dswiglu_bt192"):
    pts = []
    for K in (1024, 2048, 4096, 8192):
        if name == "swiglu_fwd":
            x, w = rnd(M, K), rnd(2 * F, K) * 0.02
            t = timeit(lambda: ext.gemm4w_swiglu(x, w, None, F))
        elif name == "nt256":
            x, w = rnd(M, K), rnd(2 * F, K) * 0.02
            t = timeit(lambda: ext.gemm4w(x, w, None, 1, False, 256, 256))
        else:
            dy, w, gu = rnd(M, K), rnd(K, F) * 0.02, rnd(M, 2 * F)
            t = timeit(lambda: ext.gemm4w_dswiglu(dy, w, gu, None))
        pts.append((K // 64, t))
        print(f"{name:14s} K={K:5d} {t:8.1f} us", flush=True)
    n = len(pts)
    sx = sum(p[0] for p in pts); sy = sum(p[1] for p in pts)
    sxx = sum(p[0] ** 2 for p in pts); sxy = sum(p[0] * p[1] for p in pts)
    b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
    a = (sy - b * sx) / n
    print(f"{name:14s} fit: {a:.1f} us fixed + {b:.3f} us per K-tile (whole grid)", flush=True)
