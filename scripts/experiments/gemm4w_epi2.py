"""Down-projection dX with the SwiGLU backward fused into the GEMM epilogue (gemm4w_dswiglu, EPI 2) vs
the plain transposed-B GEMM + the separate swiglu_bwd pass, at the Qwen3-8B MLP shape.
    M=2048 python scripts/experiments/gemm4w_epi2.py
(LIPA_GEMM4W_BM / LIPA_GEMM4W_BN force the tile of both forms.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


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
    M, F, Nw = int(os.environ.get("M", "2048")), 12288, 4096
    wd = (0.05 * torch.randn(Nw, F, device="cuda")).to(torch.bfloat16)
    gu = torch.randn(M, 2 * F, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, Nw, device="cuda").to(torch.bfloat16)
    fused = lambda: ext.gemm4w_dswiglu(dy, wd, gu)  # noqa: E731
    gemm = lambda: ext.gemm4w(dy, wd, None, 1, True)  # noqa: E731
    dh = gemm()
    act = lambda: ext.swiglu_bwd(dh, gu)  # noqa: E731
    err = (fused().float() - act().float()).abs().max().item()
    res = {}
    for _ in range(3):
        for k, fn in (("fused", fused), ("gemm", gemm), ("swiglu_bwd", act)):
            res.setdefault(k, []).append(timeit(fn))
    best = {k: min(v) for k, v in res.items()}
    print(f"M={M} F={F} Nw={Nw} BM={os.environ.get('LIPA_GEMM4W_BM', 'auto')} "
          f"BN={os.environ.get('LIPA_GEMM4W_BN', 'auto')}: fused {best['fused']:.1f} us | gemm {best['gemm']:.1f} + "
          f"swiglu_bwd {best['swiglu_bwd']:.1f} = {best['gemm'] + best['swiglu_bwd']:.1f} us | max|diff| {err:.3g}",
          flush=True)


if __name__ == "__main__":
    main()
