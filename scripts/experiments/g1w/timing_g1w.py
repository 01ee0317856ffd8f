"""Per-workgroup shader-clock cycles + 100 MHz realtime for g1w v3: effective clock and cycles per K-step."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_g1w import lib, run  # noqa: E402

lib.g1w_set_dbg.argtypes = [ctypes.c_void_p]
CASES = [("gate_up", 2048, 24576, 4096, 1256), ("dX_gu", 2048, 4096, 24576, 1256),
         ("o", 2048, 4096, 4096, 1256), ("sq8k", 8192, 8192, 8192, 1256), ("gate_up_p", 2048, 24576, 4096, 2256)]
only = os.environ.get("SHAPES")
for name, M, N, K, cfg in CASES:
    if only and name not in only.split(","):
        continue
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    nwg = (M // 256) * (N // 256)
    dbg = torch.zeros(max(nwg, 256) * 4, dtype=torch.int64, device="cuda")
    for _ in range(5):
        run(x, w, y, None, cfg, 1)
    lib.g1w_set_dbg(dbg.data_ptr())
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):
        run(x, w, y, None, cfg, 1)
    st.record()
    run(x, w, y, None, cfg, 1)
    en.record()
    torch.cuda.synchronize()
    lib.g1w_set_dbg(None)
    hb = []
    for _ in range(20):
        x @ w.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        x @ w.t()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:10s} hipblaslt {e0.elapsed_time(e1) * 100:7.1f} us", flush=True)
    d = dbg.view(-1, 4)[: (nwg if cfg < 2000 else min(nwg, 256))].cpu().double()
    cyc, rt = d[:, 0], d[:, 1] * 10.0   # ns
    clk = (cyc / rt).mean().item()      # GHz
    ksteps = K // 64 * (1 if cfg < 2000 else nwg // 256)
    print(f"{name:10s} wall {st.elapsed_time(en)*1000:7.1f} us  wg {rt.mean().item()/1000:7.1f} us (min {rt.min().item()/1000:.1f} max {rt.max().item()/1000:.1f})"
          f"  clk {clk:.3f} GHz  cyc/kstep {(cyc.mean()/ksteps).item():7.0f} (ideal 2048)", flush=True)
