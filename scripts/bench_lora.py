"""Microbenchmark of the fused LoRA branch kernels (csrc/kernels/lora.hip) at the Qwen3-8B QLoRA
bench shapes (M = 2 micro-batches x 2 x 512 tokens, r = 8, q_proj / v_proj of the fused q|k|v).
Prints µs per call and the effective HBM bandwidth of the compulsory traffic."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1000 * s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    M, H, r = 2048, 4096, 8
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, 6144, device=dev, dtype=torch.bfloat16)
    dx = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    a = torch.randn(r, H, device=dev, dtype=torch.bfloat16) * 0.02
    bq = torch.randn(r, 4096, device=dev, dtype=torch.bfloat16) * 0.02
    bv = torch.randn(r, 1024, device=dev, dtype=torch.bfloat16) * 0.02
    ext = torch.zeros(M, 16, device=dev, dtype=torch.bfloat16)
    g = torch.randn(M, r, device=dev, dtype=torch.float32)
    g2 = torch.randn(M, r, device=dev, dtype=torch.float32)
    a2 = torch.randn(r, H, device=dev, dtype=torch.bfloat16) * 0.02
    outA2 = torch.zeros(r, H, device=dev, dtype=torch.float32)
    outA = torch.zeros(r, H, device=dev, dtype=torch.float32)
    outBq = torch.zeros(4096, r, device=dev, dtype=torch.float32)
    outBv = torch.zeros(1024, r, device=dev, dtype=torch.float32)
    N = native()
    cases = {
        "proj_fwd_x_K4096_drop": (lambda: N.lora_proj(x, 0, H, a, ext[:, :r], True, 0.1, 7, 2.0), M * H * 2),
        "proj_bwd_dyq_K4096": (lambda: N.lora_proj(dy, 0, 4096, bq, None, True, 0.0, 0, 2.0), M * 4096 * 2),
        "proj_bwd_dyv_K1024": (lambda: N.lora_proj(dy, 5120, 1024, bv, None, True, 0.0, 0, 2.0), M * 1024 * 2),
        "acc_dB_q_K4096": (lambda: N.lora_acc(g, dy, 0, 4096, outBq, True, None, None, 0.0, 0, False), M * 4096 * 2),
        "acc_dB_v_K1024": (lambda: N.lora_acc(g, dy, 5120, 1024, outBv, True, None, None, 0.0, 0, False),
                           M * 1024 * 2),
        "acc_dA_dx_drop": (lambda: N.lora_acc(g, x, 0, H, outA, False, dx, a, 0.1, 7, False), 3 * M * H * 2),
        "acc_dA_dx_nodrop": (lambda: N.lora_acc(g, x, 0, H, outA, False, dx, a, 0.0, 0, False), 3 * M * H * 2),
        "acc_dA_drop_nodx": (lambda: N.lora_acc(g, x, 0, H, outA, False, None, None, 0.1, 7, False), M * H * 2),
        "dropout_fwd": (lambda: N.dropout_fwd(x, 0.1, 7), 2 * M * H * 2),
        "acc_dA_nodx": (lambda: N.lora_acc(g, x, 0, H, outA, False, None, None, 0.0, 0, False), M * H * 2),
        "pair_proj2_fwd_drop": (lambda: N.lora_proj2(x, a, a2, ext, True, 0.1, 7, 2.0, 0.1, 9, 2.0, None), M * H * 2),
    }
    import os
    only = os.environ.get("LORA_CASES")
    if only:
        cases = {k: v for k, v in cases.items() if any(o in k for o in only.split(","))}
    for name, (fn, nbytes) in cases.items():
        us = timeit(fn)
        print(json.dumps({"case": name, "us": round(us, 2), "TB_s": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
