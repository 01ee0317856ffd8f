"""gemm4w vs hipBLASLt at every GEMM of the Qwen3-8B QLoRA step (M = 2048 tokens): forward x·Wᵀ (NT)
and backward dX = dY·W (bt=True, W used as stored).  Interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24), uniform [-1, 1) operands, numerics vs an fp32 reference.
CFGS="splits:bn[:bm],…" lists the gemm4w configurations timed (0 = auto)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_in_practise_amd.ops._native import native  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1000


def main():
    ext = native()
    M = int(os.environ.get("M", "2048"))
    # (name, N_w, K_w): weight [N_w, K_w]; fwd y[M, N_w] = x[M, K_w]·Wᵀ, bwd dx[M, K_w] = dy[M, N_w]·W
    weights = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 24576, 4096), ("down", 4096, 12288)]
    cfgs = [tuple(int(v) for v in (c + ":0").split(":")[:3]) for c in os.environ.get("CFGS", "0:0").split(",")]
    tot = {}
    for name, Nw, Kw in weights:
        w = (torch.rand(Nw, Kw, device="cuda") * 2 - 1).to(torch.bfloat16)
        for kind in ("fwd", "dX"):
            if kind == "fwd":
                a = (torch.rand(M, Kw, device="cuda") * 2 - 1).to(torch.bfloat16)
                lib = lambda: a @ w.t()  # noqa: E731
                mine = lambda c: ext.gemm4w(a, w, None, c[0], False, c[1], c[2])  # noqa: E731
                ref = a.float() @ w.float().t()
                n_out, k_red = Nw, Kw
            else:
                a = (torch.rand(M, Nw, device="cuda") * 2 - 1).to(torch.bfloat16)
                lib = lambda: a @ w  # noqa: E731
                mine = lambda c: ext.gemm4w(a, w, None, c[0], True, c[1], c[2])  # noqa: E731
                ref = a.float() @ w.float()
                n_out, k_red = Kw, Nw
            errs = []
            for c in cfgs:
                y = mine(c).float()
                errs.append(f"s{c[0]}b{c[1]}m{c[2]}:{((y - ref).norm() / ref.norm()).item():.2e}")
            del ref
            res = {}
            for _ in range(3):
                res.setdefault("hipblaslt", []).append(timeit(lib))
                for c in cfgs:
                    res.setdefault(f"g4w_s{c[0]}b{c[1]}m{c[2]}", []).append(timeit(lambda: mine(c)))
            fl = 2 * M * n_out * k_red
            for k, v in res.items():
                t = min(v)
                tot[k] = tot.get(k, 0.0) + t
                print(f"{name:8s} {kind:3s} M={M:5d} N={n_out:6d} K={k_red:6d} {k:16s} {t:8.1f} us "
                      f"{fl / t / 1e6:7.1f} TF/s", flush=True)
            print(f"{name:8s} {kind:3s} relerr {' '.join(errs)}", flush=True)
    print("sum over the 8 GEMMs (one layer): " + "  ".join(f"{k} {v:.1f} us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
