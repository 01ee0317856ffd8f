"""Tiny driver for rocprofv3 --pmc: gemm4w vs hipBLASLt at one shape (default gate_up, M=2048), forward
(x·Wᵀ) and, with a 4th argument 'bt', the dX form dY·W."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

M, N, K = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 24576, 4096)))
bt = len(sys.argv) > 4 and sys.argv[4] == "bt"
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16) if bt else \
    (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
sp, bn = int(os.environ.get("SPLITS", "1")), int(os.environ.get("BN", "0"))
for _ in range(5):
    native().gemm4w(x, w, None, sp, bt, bn)
    (x @ w) if bt else (x @ w.t())
torch.cuda.synchronize()
