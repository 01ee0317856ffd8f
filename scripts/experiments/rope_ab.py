"""Time the fused q/k-norm + RoPE kernels (fwd, bwd) at the bench shape for one build of the extension:
python scripts/experiments/rope_ab.py <package root> [label].  Run the in-tree build and an ab_variants/<name> build
alternately in one gpurun call for a same-box A/B."""
import sys

import os

root = os.path.abspath(sys.argv[1])
sys.path.insert(0, root)
import torch  # noqa: E402

from llm_in_practise_amd.ops._native import native  # noqa: E402

C = native()
assert os.path.abspath(C.__file__).startswith(root), C.__file__
T, hq, hkv, d = 2048, 32, 8, 128
qkv = torch.randn(T, (hq + 2 * hkv) * d, device="cuda", dtype=torch.bfloat16)
qw = torch.ones(d, device="cuda", dtype=torch.bfloat16)
kw = torch.ones(d, device="cuda", dtype=torch.bfloat16)
pos = torch.arange(T, device="cuda", dtype=torch.float32)
inv = 1.0 / (1e6 ** (torch.arange(0, d, 2, device="cuda", dtype=torch.float32) / d))
ang = pos[:, None] * inv[None]
cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
q, k, rq, rk = C.qk_norm_rope_fwd(qkv, qw, kw, cos, sin, hq, hkv, d, 1e-6)
dq, dk = torch.randn_like(q), torch.randn_like(k)
dv = torch.randn(T, hkv * d, device="cuda", dtype=torch.bfloat16)


def timeit(fn, it=200):
    for _ in range(20):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / it)
    return best


f = timeit(lambda: C.qk_norm_rope_fwd(qkv, qw, kw, cos, sin, hq, hkv, d, 1e-6))
b = timeit(lambda: C.qk_norm_rope_bwd(dq, dk, dv, qkv, qw, kw, cos, sin, rq, rk, hq, hkv, d))
print(f"{sys.argv[2] if len(sys.argv) > 2 else root:10s} qk_norm_rope fwd {f:6.2f} us  bwd {b:6.2f} us  (T={T}, {hq}/{hkv} heads, D={d}; "
      "back-to-back launches incl. output allocation)", flush=True)
