"""A/B: one-wave-per-SIMD 256-tile GEMM (g1w.hip) vs hipBLASLt (torch.matmul), Qwen3-8B step shapes.
Interleaved rounds in one process, random uniform[-1,1) operands."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("G1W_LIB", "libg1w.so")))
lib.g1w_launch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_void_p]


def run(x, w, y, ws, bn, splits):
    M, K = x.shape
    N = w.shape[0]
    r = lib.g1w_launch(x.data_ptr(), w.data_ptr(), y.data_ptr(), ws.data_ptr() if ws is not None else None,
                       M, N, K, bn, splits, torch.cuda.current_stream().cuda_stream)
    assert r == 0, r


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
    shapes = [("qkv", 2048, 6144, 4096), ("o", 2048, 4096, 4096), ("gate_up", 2048, 24576, 4096),
              ("down", 2048, 4096, 12288), ("dX_down", 2048, 12288, 4096), ("dX_qkv", 2048, 4096, 6144),
              ("dX_gu", 2048, 4096, 24576), ("sq8k", 8192, 8192, 8192)]
    only = os.environ.get("SHAPES")
    cfgs = [tuple(int(v) for v in c.split("x")) for c in os.environ.get("CFGS", "256x1,128x1,256x2").split(",")]
    for name, M, N, K in shapes:
        if only and name not in only.split(","):
            continue
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ws = torch.empty(4 * M * N, device="cuda", dtype=torch.float32)
        ref = (x @ w.t()).float()
        fl = 2 * M * N * K
        res = {}
        ok = {}
        for bn, sp in cfgs:
            ebn = abs(bn) % 1000
            if N % ebn or (K // 64) % (2 * sp):
                continue
            y.zero_()
            run(x, w, y, ws, bn, sp)
            torch.cuda.synchronize()
            err = ((y.float() - ref).norm() / ref.norm()).item()
            ok[(bn, sp)] = err
        for rnd in range(3):
            res.setdefault("hipblaslt", []).append(timeit(lambda: x @ w.t()))
            for (bn, sp) in ok:
                res.setdefault(f"g1w_{bn}_s{sp}", []).append(timeit(lambda: run(x, w, y, ws, bn, sp)))
        for k, v in res.items():
            t = min(v)
            e = ""
            if k.startswith("g1w"):
                bn, sp = int(k.split("_")[1]), int(k.split("_s")[1])
                e = f"relerr={ok[(bn, sp)]:.2e}"
            print(f"{name:8s} M={M:5d} N={N:6d} K={K:6d} {k:12s} {t:8.1f} us {fl / t / 1e6:7.1f} TF/s {e}", flush=True)


if __name__ == "__main__":
    main()
