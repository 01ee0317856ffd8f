"""A/B: 8-phase MFMA GEMM (gemm8) vs hipBLASLt (torch.matmul) at the Qwen3-8B QLoRA shapes.

Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), random operands."""
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
              ("down", 2048, 4096, 12288), ("dX_down", 2048, 12288, 4096), ("sq4k", 4096, 4096, 4096),
              ("sq8k", 8192, 8192, 8192)]
    splits_env = [int(s) for s in os.environ.get("SPLITS", "0").split(",")]
    for name, M, N, K in shapes:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ref = x.float() @ w.float().t() if M * N * K <= 2048 * 24576 * 4096 else None
        fl = 2 * M * N * K
        res = {}
        for rnd in range(3):
            res.setdefault("hipblaslt", []).append(timeit(lambda: x @ w.t()))
            for sp in splits_env:
                res.setdefault(f"gemm8_s{sp}", []).append(timeit(lambda: ext.gemm8(x, w, None, None, None, sp)))
        err = ""
        if ref is not None:
            y = ext.gemm8(x, w, None, None, None, 0).float()
            err = f"relerr={((y - ref).norm() / ref.norm()).item():.2e}"
        for k, v in res.items():
            t = min(v)
            print(f"{name:8s} M={M:5d} N={N:6d} K={K:6d} {k:12s} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s {err}", flush=True)


if __name__ == "__main__":
    main()
