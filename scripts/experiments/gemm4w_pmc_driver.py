"""Tiny driver for rocprofv3 --pmc: gemm4w vs hipBLASLt at one shape (default gate_up, M=2048)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 24576, 4096)))
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
for _ in range(5):
    native().gemm4w(x, w, None, 1)
    x @ w.t()
torch.cuda.synchronize()
