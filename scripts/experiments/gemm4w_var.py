"""gemm4w diagnostic / schedule variants (LIPA_GEMM4W_VAR read once per process, so one process per
variant): timing at the gate|up and 8k shapes, relative error vs an fp32 reference (ablation variants
1-7 are wrong by design)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

var = os.environ.get('LIPA_GEMM4W_VAR', '0')
for M, N, K in ((2048, 24576, 4096), (8192, 8192, 8192), (1000, 1536, 1024)):
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = native().gemm4w(x, w, None, 1).float()
    ref = x.float() @ w.float().t()
    err = ((y - ref).norm() / ref.norm()).item()
    del ref, y
    for _ in range(3):
        native().gemm4w(x, w, None, 1)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for r in range(3):
        st.record()
        for _ in range(10):
            native().gemm4w(x, w, None, 1)
        en.record()
        torch.cuda.synchronize()
        best = min(best, st.elapsed_time(en) / 10 * 1000)
    print(f"var={var} M={M} N={N} K={K} {best:.1f} us {2 * M * N * K / best / 1e6:.0f} TF/s relerr={err:.2e}",
          flush=True)
