"""Isolation of the plain NF4-code (W4) gemm4w calls the unfused SwiGLU MLP makes in LIPA_NF4_GEMM=w4 mode,
one call per process (argv[1]): gu_fwd = x·Wgu^T (NT, N = 24576, K = 4096), down_dx = dy·Wdown (BT,
N = 12288, K = 4096), down_fwd (NT + residual, N = 4096, K = 12288), gu_dx (BT, N = 4096, K = 24576),
each against gemm4w on the expanded bf16 weight."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_in_practise_amd.ops._native import native  # noqa: E402
from llm_in_practise_amd.quant.nf4 import quantize_nf4  # noqa: E402

ext = native()
M, d, f = 2048, 4096, 12288
case = sys.argv[1]
if case.startswith("lorafwd"):   # the q|k|v forward with the LoRA B term in the prologue, NF4 codes
    Mx = int(case.split("_")[1])
    q = quantize_nf4((0.02 * torch.randn(6144, d, device="cuda")).to(torch.bfloat16), 64, True)
    codes, sc = q.g4w_pack()
    wd = ext.nf4_dequant_fast(q.codes, q.gemv_scales(), 6144, d)
    x = (torch.rand(Mx, d, device="cuda") * 2 - 1).to(torch.bfloat16)
    xa = (torch.randn(Mx, 32, device="cuda") * 0.1).bfloat16()
    bs = [(torch.randn(4096, 8, device="cuda") * 0.05).bfloat16(), (torch.randn(1024, 8, device="cuda") * 0.05).bfloat16()]
    y4 = ext.gemm4w_lora(x, codes, sc, 6144, None, xa, bs, [0, 5120], [0, 8], [None, None])
    torch.cuda.synchronize()
    y = ext.gemm4w_lora(x, wd, None, 0, None, xa, bs, [0, 5120], [0, 8], [None, None])
    torch.cuda.synchronize()
    print(case, "max|diff|", (y4.float() - y.float()).abs().max().item(), flush=True)
    sys.exit(0)
if case.startswith("loradx"):   # the q|k|v dX with the masked LoRA dx term in the prologue, NF4 codes (w4 mode)
    Mx = int(case.split("_")[1]) if "_" in case else M
    q = quantize_nf4((0.02 * torch.randn(6144, d, device="cuda")).to(torch.bfloat16), 64, True)
    codes, sc = q.g4w_pack()
    wd = ext.nf4_dequant_fast(q.codes, q.gemv_scales(), 6144, d)
    dy = (torch.rand(Mx, 6144, device="cuda") * 2 - 1).to(torch.bfloat16)
    gs = [torch.randn(Mx, 8, device="cuda"), torch.randn(Mx, 8, device="cuda")]
    As = [(torch.randn(8, d, device="cuda") * 0.05).bfloat16() for _ in range(2)]
    masks = torch.randint(0, 256, (2, Mx, d // 8), dtype=torch.uint8, device="cuda")
    ref = dy.float() @ wd.float()
    for b in range(2):
        t = gs[b] @ As[b].float()
        sh = torch.arange(8, device="cuda", dtype=torch.uint8)
        keep = ((masks[b][..., None] >> sh) & 1).bool().reshape(Mx, d)
        ref += t * keep / 0.9
    for bm in (128, 256):
        for bn in (128, 256):
            y4 = ext.gemm4w_loradx(dy, codes, sc, d, gs, As, masks, [0.1, 0.1], bn, bm)
            torch.cuda.synchronize()
            y = ext.gemm4w_loradx(dy, wd, None, 0, gs, As, masks, [0.1, 0.1], bn, bm)
            torch.cuda.synchronize()
            print(case, f"bm={bm} bn={bn} w4-vs-bf16 max|diff|", (y4.float() - y.float()).abs().max().item(),
                  "rel vs fp32: w4", ((y4.float() - ref).norm() / ref.norm()).item(),
                  "bf16", ((y.float() - ref).norm() / ref.norm()).item(), flush=True)
    sys.exit(0)
R, C, bt, resid = {"gu_fwd": (2 * f, d, False, False), "down_dx": (d, f, True, False),
                   "down_fwd": (d, f, False, True), "gu_dx": (2 * f, d, True, False)}[case]
q = quantize_nf4((0.02 * torch.randn(R, C, device="cuda")).to(torch.bfloat16), 64, True)
codes, sc = q.g4w_pack()
wd = ext.nf4_dequant_fast(q.codes, q.gemv_scales(), R, C)
K, N = (R, C) if bt else (C, R)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
res = torch.randn(M, N, device="cuda").to(torch.bfloat16) if resid else None
y4 = ext.gemm4w(x, codes, res, 0, bt, 0, 0, sc, N)
torch.cuda.synchronize()
y = ext.gemm4w(x, wd, res, 0, bt)
torch.cuda.synchronize()
print(case, "max|diff|", (y4.float() - y.float()).abs().max().item(), "rel", ((y4.float() - y.float()).norm() / y.float().norm()).item(), flush=True)
