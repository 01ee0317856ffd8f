"""A/B: one-wave-per-SIMD AGPR GEMM (gemm4w) vs hipBLASLt (torch.matmul) at the Qwen3-8B
QLoRA step shapes.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24),
uniform [-1, 1) operands; numerics vs an fp32 reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    shapes = [("qkv", 2048, 6144, 4096), ("o", 2048, 4096, 4096), ("gate_up", 2048, 24576, 4096),
              ("down", 2048, 4096, 12288), ("dX_down", 2048, 12288, 4096), ("odd", 1000, 1536, 1024),
              ("sq8k", 8192, 8192, 8192)]
    if os.environ.get("SHAPES"):
        keep = os.environ["SHAPES"].split(",")
        shapes = [s for s in shapes if s[0] in keep]
    splits = [int(s) for s in os.environ.get("SPLITS", "0").split(",")]
    for name, M, N, K in shapes:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        r = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        fl = 2 * M * N * K
        ref = (x.float() @ w.float().t() + r.float()) if M * N <= 2048 * 24576 else None
        errs = []
        if ref is not None:
            for sp in splits:
                y = ext.gemm4w(x, w, r, sp).float()
                errs.append(f"s{sp}:{((y - ref).norm() / ref.norm()).item():.2e}")
        res = {}
        for rnd in range(3):
            res.setdefault("hipblaslt", []).append(timeit(lambda: x @ w.t()))
            for sp in splits:
                res.setdefault(f"gemm4w_s{sp}", []).append(timeit(lambda: ext.gemm4w(x, w, None, sp)))
        for k, v in res.items():
            t = min(v)
            print(f"{name:8s} M={M:5d} N={N:6d} K={K:6d} {k:12s} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s", flush=True)
        print(f"{name:8s} relerr(+residual) {' '.join(errs)}", flush=True)


if __name__ == "__main__":
    main()
