"""Run-to-run check of the attention backward at one shape: the kernels use no atomics, so dQ / dK / dV must be
bit-identical over repeated calls.  Prints the number of calls whose outputs differ from the first call.

    python scripts/experiments/attn_bwd_repeat.py [--B 4 --S 512 --hq 8 --hkv 4 --iters 200 --fused]
(--fused: q / k / v as column views of one fused [T, (hq + 2 hkv)·d] projection, as the model calls it)
"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=512)
    ap.add_argument("--hq", type=int, default=8)
    ap.add_argument("--hkv", type=int, default=4)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--fused", action="store_true")
    a = ap.parse_args()
    B, S, hq, hkv, d = a.B, a.S, a.hq, a.hkv, 128
    ext = native()
    T = B * S
    torch.manual_seed(0)
    if a.fused:
        qkv = torch.randn(T, (hq + 2 * hkv) * d, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[:, :hq * d], qkv[:, hq * d:(hq + hkv) * d], qkv[:, (hq + hkv) * d:]
    else:
        q = torch.randn(T, hq * d, device="cuda").to(torch.bfloat16)
        kv = torch.randn(T, 2 * hkv * d, device="cuda").to(torch.bfloat16)
        k, v = kv[:, :hkv * d], kv[:, hkv * d:]
    scale = 1 / math.sqrt(d)
    o, lse = ext.attn_fwd(q, k, v, None, B, S, hq, hkv, d, True, scale)
    do = torch.randn_like(o)
    ref = [t.clone() for t in ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, d, True, scale, 0.0, 0)]
    bad = [0, 0, 0]
    first = None
    for i in range(a.iters):
        out = ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, d, True, scale, 0.0, 0)
        for j in range(3):
            if not torch.equal(out[j], ref[j]):
                bad[j] += 1
                if first is None:
                    diff = (out[j].float() - ref[j].float()).abs()
                    idx = int(diff.argmax())
                    first = (i, "dq dk dv".split()[j], float(diff.max()), idx // out[j].shape[1], idx % out[j].shape[1],
                             bool(torch.isfinite(out[j]).all()))
    print(f"shape {[B, S, hq, hkv, d]} fused={a.fused} iters {a.iters}: differing calls dq {bad[0]} dk {bad[1]} "
          f"dv {bad[2]}; first {first}", flush=True)


if __name__ == "__main__":
    main()
