"""Driver for rocprofv3 --pmc passes: gemm4w on a bf16 weight and on the same weight's NF4 codes (W4),
one shape.  usage: pmc_gemm4w_w4.py M N K [bt] ; env BN / BM force the tile (0 = cost model)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.nf4 import quantize_nf4  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
bt = len(sys.argv) > 4 and sys.argv[4] == "bt"
R, C = (K, N) if bt else (N, K)
bn, bm = int(os.environ.get("BN", "0")), int(os.environ.get("BM", "0"))
q = quantize_nf4((0.02 * torch.randn(R, C, device="cuda")).to(torch.bfloat16), 64, True)
codes, sc = q.g4w_pack()
wd = native().nf4_dequant_fast(q.codes, q.gemv_scales(), R, C)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
for _ in range(8):
    native().gemm4w(x, wd, None, 0, bt, bn, bm)
    native().gemm4w(x, codes, None, 0, bt, bn, bm, sc, N)
torch.cuda.synchronize()
