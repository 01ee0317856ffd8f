"""Phase timeline of the D = 128 dK/dV kernel (attn_bwd_dkv128_k, TRACE build) at one shape.

Every wave's lane 0 stamps s_memtime at the loop's phase boundaries (top, after the barrier, after the S / dP
+ softmax-gradient phase) and s_memrealtime at start / end; this script prints per-workgroup durations, the
dispatch skew, how workgroups share CUs, and the critical workgroup's per-iteration phase split.

    python scripts/experiments/attn_dkv_trace.py [--B 4 --S 512]
"""
import argparse
import collections
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
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    a = ap.parse_args()
    B, S, hq, hkv, d = a.B, a.S, a.hq, a.hkv, 128
    ext = native()
    T = B * S
    torch.manual_seed(0)
    q = torch.randn(T, hq * d, device="cuda").to(torch.bfloat16)
    kv = torch.randn(T, 2 * hkv * d, device="cuda").to(torch.bfloat16)
    k, v = kv[:, :hkv * d], kv[:, hkv * d:]
    scale = 1 / math.sqrt(d)
    o, lse = ext.attn_fwd(q, k, v, None, B, S, hq, hkv, d, True, scale)
    do = torch.randn_like(o)
    for _ in range(5):
        ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, d, True, scale, 0.0, 0)
    nb = (S + 63) // 64
    nwg = nb * hkv * B
    buf = torch.zeros(nwg * 8 * 264, dtype=torch.int64, device="cuda")
    ext.attn_set_trace(buf)
    torch.cuda.synchronize()
    ext.attn_bwd(do, q, k, v, o, lse, None, B, S, hq, hkv, d, True, scale, 0.0, 0)
    torch.cuda.synchronize()
    ext.attn_set_trace(None)
    t = buf.view(nwg, 8, 264).cpu().numpy().astype("int64")

    rt0 = t[:, 0, 6].min()
    rows = []
    for wg in range(nwg):
        w0 = t[wg, 0]
        hw_id, xcc = int(w0[0]) & 0xFFFFFFFF, int(w0[1]) & 0xF
        cu, se = (hw_id >> 8) & 0xF, (hw_id >> 13) & 0x7
        unit, n_it = int(w0[2]) & 0xFFFFFFFF, int(w0[3])
        rows.append(dict(wg=wg, xcc=xcc, se=se, cu=cu, kb=unit // 2, n_it=n_it,
                         start_us=(w0[6] - rt0) / 100.0, end_us=(w0[7] - rt0) / 100.0,
                         cyc=int(w0[5] - w0[4])))
    span = max(r["end_us"] for r in rows)
    print(f"shape B={B} S={S} hq={hq} hkv={hkv}: {nwg} workgroups, span {span:.1f} us (s_memrealtime, 10 ns ticks)")
    starts = sorted(r["start_us"] for r in rows)
    print(f"start skew: first {starts[0]:.2f} median {starts[len(starts)//2]:.2f} last {starts[-1]:.2f} us")
    occ = collections.Counter((r["xcc"], r["se"], r["cu"]) for r in rows)
    print(f"distinct (xcc, se, cu): {len(occ)}; workgroups per CU histogram: {sorted(collections.Counter(occ.values()).items())}")
    by_it = collections.defaultdict(list)
    for r in rows:
        by_it[r["n_it"]].append(r)
    print("n_it  count  mean_dur_us  max_dur_us  mean_cyc/it  mean_end_us")
    for n in sorted(by_it):
        rs = by_it[n]
        dur = [r["end_us"] - r["start_us"] for r in rs]
        cpi = [r["cyc"] / max(n, 1) for r in rs]
        print(f"{n:4d} {len(rs):6d} {sum(dur)/len(dur):12.2f} {max(dur):11.2f} {sum(cpi)/len(cpi):12.0f} "
              f"{sum(r['end_us'] for r in rs)/len(rs):12.2f}")
    crit = max(rows, key=lambda r: r["end_us"])
    print(f"critical wg {crit['wg']}: kb {crit['kb']} n_it {crit['n_it']} start {crit['start_us']:.2f} "
          f"end {crit['end_us']:.2f} us, {crit['cyc']} memtime cycles")
    print("per-iteration memtime cycles for its 8 waves: wait+barrier | S/dP+softmax | dK/dV issue->next top")
    for w in range(8):
        ev = t[crit["wg"], w]
        n = int(ev[3])
        parts = []
        for it in range(min(n, 64)):
            e0, e1, e2 = ev[8 + 4 * it], ev[8 + 4 * it + 1], ev[8 + 4 * it + 2]
            nxt = ev[8 + 4 * (it + 1)] if it + 1 < n else ev[5]
            if e2:
                parts.append(f"{e1 - e0}|{e2 - e1}|{nxt - e2}")
            else:
                parts.append(f"{e1 - e0}|skip|{nxt - e1}")
        print(f" w{w}: start->loop {ev[8] - ev[4]}  " + "  ".join(parts))


if __name__ == "__main__":
    main()
