"""gemm4w tile / split sweep at the Qwen3-8B step shapes (M = 2048, or $M): every (BN, BM, splits) the kernel
instantiates, interleaved rounds in one process, min over rounds; the cost model's pick is 'auto'."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1000


ext = native()
M = int(os.environ.get("M", "2048"))
# (name, A cols (K of the GEMM), W shape as stored, bt)
ops = [("gate_up_dX", 24576, (24576, 4096), True), ("down_fwd", 12288, (4096, 12288), False),
       ("qkv_fwd", 4096, (6144, 4096), False), ("qkv_dX", 6144, (6144, 4096), True),
       ("o_fwd", 4096, (4096, 4096), False), ("o_dX", 4096, (4096, 4096), True)]
if os.environ.get("OPS"):
    ops = [o for o in ops if o[0] in os.environ["OPS"].split(",")]
cfgs = [(0, 0, 0)] + [(bn, bm, sp) for bm in (256, 128) for bn in (256, 192, 128) for sp in (1, 2, 4)]
for name, K, wshape, bt in ops:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (0.02 * (torch.rand(*wshape, device="cuda") * 2 - 1)).to(torch.bfloat16)
    N = wshape[1] if bt else wshape[0]
    res = {}
    for _ in range(3):
        for bn, bm, sp in cfgs:
            if bn == 192 and bt and bm == 128:
                continue
            try:
                t = timeit(lambda: ext.gemm4w(a, w, None, sp, bt, bn, bm))
            except RuntimeError:
                continue
            res.setdefault((bn, bm, sp), []).append(t)
    fl = 2 * M * N * K
    best = sorted(res.items(), key=lambda kv: min(kv[1]))
    auto = min(res[(0, 0, 0)])
    line = " ".join(f"{bn}x{bm}s{sp}:{min(v):.1f}" for (bn, bm, sp), v in best[:6])
    print(f"{name:11s} N={N:6d} K={K:6d} auto {auto:7.1f} us ({fl / auto / 1e6:6.0f} TF/s) | best: {line}", flush=True)
