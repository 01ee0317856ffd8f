import sys, torch
sys.path.insert(0, "/root/repo") if False else None
import os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from llm_in_practise_amd.ops._native import native
from llm_in_practise_amd.ops.gemm import head_logits
w = (0.02 * torch.randn(151936, 4096, device="cuda")).to(torch.bfloat16)
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return 1000 * s.elapsed_time(e) / it
for M in (1, 4, 16, 64, 256):
    x = torch.randn(M, 4096, device="cuda").to(torch.bfloat16)
    a = t(lambda: head_logits(x, w)); b = t(lambda: x @ w.t())
    print(f"M={M:4d} head_logits(gemm4w) {a:8.1f} us   torch matmul {b:8.1f} us")
