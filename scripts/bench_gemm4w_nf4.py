"""NF4 codes fed straight into gemm4w (W4) vs gemm4w on the bf16 expansion vs the round-3 default
(nf4_dequant_fast + gemm4w on the copy), at every frozen-base GEMM of the Qwen3-8B QLoRA step:
forward x·Wᵀ (NT, gate|up with the SwiGLU epilogue) and dX dY·W (BT, down with the SwiGLU-backward
epilogue), M = 2048 (the fused-GA headline) and M = 1024 (the faithful micro-batch).  Interleaved
rounds in one process; min over rounds.  CFGS="bn:bm,…" adds forced W4 tile configs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.nf4 import quantize_nf4  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1000


def main():
    ext = native()
    Ms = [int(m) for m in os.environ.get("MS", "2048,1024").split(",")]
    cfgs = [tuple(int(v) for v in c.split(":")) for c in os.environ.get("CFGS", "").split(",") if c]
    d, f, qkv = 4096, 12288, 6144
    # (name, W rows, W cols, bt, epi)
    gemms = [("qkv", qkv, d, False, 0), ("o", d, d, False, 0), ("gate_up", 2 * f, d, False, 1),
             ("down", d, f, False, 0), ("qkv_dX", qkv, d, True, 0), ("o_dX", d, d, True, 0),
             ("gate_up_dX", 2 * f, d, True, 0), ("down_dX", d, f, True, 2)]
    if os.environ.get("SHAPES"):
        keep = os.environ["SHAPES"].split(",")
        gemms = [g for g in gemms if g[0] in keep]
    tot = {}
    for name, R, C, bt, epi in gemms:
        q = quantize_nf4((0.02 * torch.randn(R, C, device="cuda")).to(torch.bfloat16), 64, True)
        codes, sc = q.g4w_pack()
        wd = ext.nf4_dequant_fast(q.codes, q.gemv_scales(), R, C)
        for M in Ms:
            K = R if bt else C
            N = C if bt else R
            a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            fl = 2 * M * N * K
            if epi == 1:
                F_ = R // 2
                runs = {"bf16": lambda: ext.gemm4w_swiglu(a, wd),
                        "deq+bf16": lambda: (ext.nf4_dequant_fast(q.codes, q.gemv_scales(), R, C),
                                             ext.gemm4w_swiglu(a, wd)),
                        "w4": lambda: ext.gemm4w_swiglu(a, codes, sc, F_)}
            elif epi == 2:
                gu = torch.randn(M, 2 * C, device="cuda").to(torch.bfloat16)
                runs = {"bf16": lambda: ext.gemm4w_dswiglu(a, wd, gu),
                        "deq+bf16": lambda: (ext.nf4_dequant_fast(q.codes, q.gemv_scales(), R, C),
                                             ext.gemm4w_dswiglu(a, wd, gu)),
                        "w4": lambda: ext.gemm4w_dswiglu(a, codes, gu, sc)}
            else:
                runs = {"bf16": lambda: ext.gemm4w(a, wd, None, 0, bt),
                        "deq+bf16": lambda: (ext.nf4_dequant_fast(q.codes, q.gemv_scales(), R, C),
                                             ext.gemm4w(a, wd, None, 0, bt)),
                        "w4": lambda: ext.gemm4w(a, codes, None, 0, bt, 0, 0, sc, N)}
                for bn, bm in cfgs:
                    runs[f"w4_{bn}x{bm}"] = (lambda bn=bn, bm=bm: ext.gemm4w(a, codes, None, 0, bt, bn, bm, sc, N))
            res = {}
            for _ in range(3):
                for k, fn in runs.items():
                    res.setdefault(k, []).append(timeit(fn))
            line = f"{name:11s} M={M:5d} N={N:6d} K={K:6d}"
            for k, v in res.items():
                t = min(v)
                tot[(M, k)] = tot.get((M, k), 0.0) + t
                line += f"  {k} {t:7.1f} us {fl / t / 1e6:6.0f} TF/s"
            line += f"  w4/bf16 {min(res['w4']) / min(res['bf16']):.3f}"
            print(line, flush=True)
    for (M, k), t in sorted(tot.items()):
        print(f"sum M={M} {k:10s} {t:8.1f} us per layer", flush=True)


if __name__ == "__main__":
    main()
