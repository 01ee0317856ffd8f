"""Probe of the q+v LoRA forward kernels at the bench shape (M = 2048 tokens, K = 4096, r = 8 + 8):
lora_proj2 with / without the stored keep bits and with / without dropout.  µs per call, cold-L2
variant (a 512 MB buffer is touched between calls, as the GEMMs do inside the step)."""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, iters=50, flush=None):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    if flush is None:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return 1000 * s.elapsed_time(e) / iters
    for _ in range(iters):
        flush.add_(1)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        tot += s.elapsed_time(e)
    return 1000 * tot / iters


def main():
    dev = torch.device("cuda")
    M, H, r = 2048, 4096, 8
    N = native()
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    a0 = torch.randn(r, H, device=dev, dtype=torch.bfloat16) * 0.02
    a1 = torch.randn(r, H, device=dev, dtype=torch.bfloat16) * 0.02
    ext = torch.zeros(M, 2 * r, device=dev, dtype=torch.bfloat16)
    masks = torch.empty(2, M, H // 8, device=dev, dtype=torch.uint8)
    flush = torch.zeros(128 << 20, device=dev, dtype=torch.float32)
    impl = os.environ.get("LIPA_PROJ2_IMPL")
    cases = {
        "proj2_drop_mask": lambda: N.lora_proj2(x, a0, a1, ext, True, 0.1, 7, 2.0, 0.1, 9, 2.0, masks),
        "proj2_drop": lambda: N.lora_proj2(x, a0, a1, ext, True, 0.1, 7, 2.0, 0.1, 9, 2.0, None),
        "proj2_nodrop": lambda: N.lora_proj2(x, a0, a1, ext, True, 0.0, 7, 2.0, 0.0, 9, 2.0, None),
    }
    for name, fn in cases.items():
        hot = timeit(fn)
        cold = timeit(fn, iters=20, flush=flush)
        print(json.dumps({"impl": impl, "case": name, "us_hot": round(hot, 2), "us_cold": round(cold, 2),
                          "TB_s_hot": round(M * H * 2 / hot / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
