"""Locate non-finite outputs of gemm4w_loradx (the LoRA dx term computed in the dX GEMM prologue)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402

ext = native()
DEV = "cuda"


def run(M, Nk, K, r, nbr, gz=False, az=False, mask=None):
    torch.manual_seed(11)
    dy = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (0.05 * torch.randn(K, Nk, device=DEV)).to(torch.bfloat16)
    gs = [torch.zeros(M, r, device=DEV) if gz else torch.randn(M, r, device=DEV) for _ in range(nbr)]
    As = [(torch.zeros if az else torch.randn)(r, Nk, device=DEV).mul(0.05).to(torch.bfloat16) for _ in range(nbr)]
    if mask is None:
        masks = torch.randint(0, 256, (nbr, M, Nk // 8), device=DEV, dtype=torch.uint8)
    else:
        masks = torch.full((nbr, M, Nk // 8), mask, device=DEV, dtype=torch.uint8)
    dx = ext.gemm4w_loradx(dy, w, None, 0, gs, As, masks, [0.1, 0.05][:nbr])
    base = ext.gemm4w(dy, w, None, 0, True)
    bad = ~torch.isfinite(dx.float())
    d = (dx.float() - base.float()).abs()
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print(f"M={M} Nk={Nk} K={K} r={r} nbr={nbr} gz={gz} az={az} mask={mask}: nonfinite={int(bad.sum())} "
          f"rows={rows[:8].tolist()}..{len(rows)} cols={cols[:8].tolist()}..{len(cols)} "
          f"max|dx-base|(finite)={float(d[~bad].max()) if (~bad).any() else -1:.3f}", flush=True)


for args in [(2048, 4096, 6144, 8, 2), (2048, 4096, 6144, 8, 1), (2048, 4096, 6144, 8, 2, True),
             (2048, 4096, 6144, 8, 2, False, True), (2048, 4096, 6144, 8, 2, False, False, 0),
             (2048, 4096, 6144, 8, 2, False, False, 255), (300, 640, 1024, 16, 2), (512, 1152, 256, 8, 2)]:
    run(*args)
