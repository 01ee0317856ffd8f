"""Multi-LoRA decode cost vs the number of LOADED adapters (verdict r2 #7): the segment kernel
(mlora_apply) against the round-2 masked form (x·A_allᵀ ⊙ S[ids]) · B_allᵀ, one Qwen3-8B q|k|v-sized
projection (K = 4096, N = 6144, rank 16), 64 decode rows all on adapter 1, with 1 and 8 adapters loaded."""
import os
import struct
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def run(n_adapters, T=64, K=4096, N=6144, r=16):
    R = r * n_adapters
    A = (0.02 * torch.randn(R, K, device="cuda")).to(torch.bfloat16)
    B = (0.02 * torch.randn(N, R, device="cuda")).to(torch.bfloat16)
    seg = [[0, 0, 0]] + [[i * r, r, struct.unpack("<i", struct.pack("<f", 2.0))[0]] for i in range(n_adapters)]
    seg = torch.tensor(seg, dtype=torch.int32, device="cuda")
    cs = torch.zeros(n_adapters + 1, R, device="cuda", dtype=torch.bfloat16)
    for i in range(n_adapters):
        cs[i + 1, i * r:(i + 1) * r] = 2.0
    ids = torch.ones(T, dtype=torch.long, device="cuda")
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    y = torch.zeros(T, N, device="cuda", dtype=torch.bfloat16)

    def seg_k():
        native().mlora_apply(x, A, B, ids, seg, y, 0)

    def masked():
        y.add_(((x @ A.t()) * cs.index_select(0, ids)) @ B.t())

    out = {}
    for name, fn in (("segment", seg_k), ("masked", masked)):
        for _ in range(5):
            fn()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(50):
            fn()
        en.record()
        torch.cuda.synchronize()
        out[name] = st.elapsed_time(en) / 50 * 1000
    return out


for n in (1, 2, 8):
    r = run(n)
    print(f"adapters loaded={n}: segment kernel {r['segment']:.1f} us   masked torch form {r['masked']:.1f} us",
          flush=True)
