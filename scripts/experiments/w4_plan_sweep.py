"""Tile / split sweep of the affine-int4 gemm4w (W4 = 2) at decode-batch row counts vs the bf16 gemm4w plan:
python scripts/experiments/w4_plan_sweep.py.  Qwen3-8B projection shapes; one process, min of 5 x 20 launches."""
import torch

from llm_in_practise_amd.ops._native import native
from llm_in_practise_amd.quant.int4 import quantize_rtn

C = native()
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (24576, 4096), "down": (4096, 12288)}


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / it)
    return best


torch.manual_seed(0)
for M in (128, 256):
    for name, (N, K) in SHAPES.items():
        w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
        q = quantize_rtn(w, 128)
        codes, sc, zr = q.g4w_pack()
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        tb = timeit(lambda: C.gemm4w(x, w, None, 0, False, 0, 0, None, 0, None))
        ref = C.gemm4w(x, codes, None, 0, False, 0, 0, sc, N, zr)
        auto = timeit(lambda: C.gemm4w(x, codes, None, 0, False, 0, 0, sc, N, zr))
        res = []
        for bm in (256, 128):
            for bn in (256, 128):
                for sp in (1, 2, 4):
                    if K // 64 // sp < 8:
                        continue
                    y = C.gemm4w(x, codes, None, sp, False, bn, bm, sc, N, zr)
                    err = ((y.float() - ref.float()).norm() / ref.float().norm()).item()
                    t = timeit(lambda: C.gemm4w(x, codes, None, sp, False, bn, bm, sc, N, zr))
                    res.append((t, f"{bm}x{bn}s{sp}", err))
        res.sort()
        best = " ".join(f"{n}:{t:.1f}" for t, n, _ in res[:4])
        print(f"M={M:4d} {name:8s} bf16 {tb:6.1f} us | int4 auto {auto:6.1f} us | best {best} | max relerr vs auto "
              f"{max(e for _, _, e in res):.1e}", flush=True)
