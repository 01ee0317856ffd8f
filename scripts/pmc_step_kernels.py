"""Driver for rocprofv3 --pmc passes over the kernels the Qwen3-8B QLoRA step ships, at its shapes
(M = 2048 tokens, bf16): the gemm4w variants the cost model picks (q|k|v and o forward / dX, gate|up
forward with the SwiGLU epilogue, down forward (split-K) and its dX with the SwiGLU-backward epilogue,
gate|up dX (split-K) + splitk_sum) and the flash-attention forward / dQ / dK-dV kernels at
[B 4, S 512, hq 32, hkv 8, d 128].  8 repetitions each; pmc_summary.py averages per kernel."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

ext = native()
M, d, f = 2048, 4096, 12288
rnd = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
w_qkv, w_o, w_gu, w_d = rnd(6144, d) * 0.02, rnd(d, d) * 0.02, rnd(2 * f, d) * 0.02, rnd(d, f) * 0.02
x, h = rnd(M, d), rnd(M, f)
dy_qkv, dy_d, dy_gu = rnd(M, 6144), rnd(M, d), rnd(M, 2 * f)
gu = rnd(M, 2 * f)
B, S, hq, hkv, hd = 4, 512, 32, 8, 128
q = rnd(B * S, hq * hd)
kv = rnd(B * S, 2 * hkv * hd)
k, v = kv[:, :hkv * hd], kv[:, hkv * hd:]
o, lse = ext.attn_fwd(q, k, v, None, B, S, hq, hkv, hd, True, 1 / math.sqrt(hd))
do = rnd(B * S, hq * hd)
for _ in range(8):
    ext.gemm4w(x, w_qkv, None, 0, False)                 # q|k|v forward
    ext.gemm4w(dy_qkv, w_qkv, None, 0, True)             # q|k|v dX
    ext.gemm4w(x, w_o, x, 0, False)                      # o forward (+ residual)
    ext.gemm4w(dy_d, w_o, None, 0, True)                 # o dX
    ext.gemm4w_swiglu(x, w_gu, None, f)                  # gate|up forward + SwiGLU epilogue
    ext.gemm4w(h, w_d, x, 0, False)                      # down forward (split-K + splitk_sum)
    ext.gemm4w_dswiglu(dy_d, w_d, gu, None)              # down dX + SwiGLU-backward epilogue
    ext.gemm4w(dy_gu, w_gu, None, 0, True)               # gate|up dX (split-K + splitk_sum)
    ext.attn_fwd(q, k, v, None, B, S, hq, hkv, hd, True, 1 / math.sqrt(hd))
    ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, hd, True, 1 / math.sqrt(hd), 0.0, 0)
torch.cuda.synchronize()
