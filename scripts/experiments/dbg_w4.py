import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native
from llm_in_practise_amd.quant.int4 import quantize_rtn
nat = native()
torch.manual_seed(2)
for (N, K) in [(6144, 4096), (4096, 4096), (4096, 12288)]:
    w4 = quantize_rtn(torch.randn(N, K, device="cuda") * 0.02, 128, False)
    s, b = w4.gemv_tables()
    wd = w4.dequantize()
    for M in [2, 16, 17, 32, 33, 64]:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        ref = x.float() @ wd.t()
        ys = [nat.gemm_w4_skinny(x, w4.codes, s, b, N, 128, None).float() for _ in range(3)]
        for _ in range(20):
            nat.gemm_w4_skinny(x, w4.codes, s, b, N, 128, None)
        ys.append(nat.gemm_w4_skinny(x, w4.codes, s, b, N, 128, None).float())
        errs = [round(((y - ref).norm() / ref.norm()).item(), 4) for y in ys]
        same = [bool(torch.equal(ys[0], y)) for y in ys[1:]]
        d = (ys[-1] - ref).abs() > 0.05 * ref.abs().max()
        rows = d.any(1).nonzero().flatten().tolist()
        cols = d.any(0).nonzero().flatten()
        print(N, K, M, "errs", errs, "deterministic", same, "bad rows", rows[:10], "ncols", cols.numel(),
              "col blocks", sorted(set((cols // 16).tolist()))[:12], flush=True)
