"""Isolate the transposed-B (dX) cost: the same M×N×K through gemm4w NT (w [N, K]) and BT (w [K, N]),
both tile widths, interleaved rounds; default shape = gate|up dX at M = 2048."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 4096, 24576)))
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w_nt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w_bt = w_nt.t().contiguous()
ref = x.float() @ w_nt.float().t()
cfgs = [("nt", w_nt, False, 2, 256), ("bt", w_bt, True, 2, 256), ("nt", w_nt, False, 1, 128), ("bt", w_bt, True, 1, 128)]
for name, w, bt, sp, bn in cfgs:
    y = native().gemm4w(x, w, None, sp, bt, bn).float()
    print(f"{name} s{sp} b{bn} relerr {((y - ref).norm() / ref.norm()).item():.2e}", flush=True)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {}
for _ in range(3):
    for name, w, bt, sp, bn in cfgs:
        for _ in range(2):
            native().gemm4w(x, w, None, sp, bt, bn)
        st.record()
        for _ in range(10):
            native().gemm4w(x, w, None, sp, bt, bn)
        en.record()
        torch.cuda.synchronize()
        res.setdefault(f"{name} s{sp} b{bn}", []).append(st.elapsed_time(en) / 10 * 1000)
for k, v in res.items():
    print(f"M={M} N={N} K={K} {k:12s} {min(v):8.1f} us {2 * M * N * K / min(v) / 1e6:7.1f} TF/s", flush=True)
