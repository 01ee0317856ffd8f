"""rocprofv3 --pmc driver: g1w configs + hipBLASLt on one shape (SHAPE=M,N,K; CFGS like bench_g1w)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_g1w import run  # noqa: E402

M, N, K = (int(v) for v in os.environ.get("SHAPE", "2048,24576,4096").split(","))
cfgs = [tuple(int(v) for v in c.split("x")) for c in os.environ.get("CFGS", "256x1").split(",")]
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
ws = torch.empty(4 * M * N, device="cuda", dtype=torch.float32)
for _ in range(3):
    x @ w.t()
    for bn, sp in cfgs:
        run(x, w, y, ws, bn, sp)
torch.cuda.synchronize()
