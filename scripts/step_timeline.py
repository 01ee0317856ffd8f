#!/usr/bin/env python3
"""GPU busy vs wall time per training step from a rocprofv3 kernel trace.

Steps are delimited by the optimizer kernel (adamw / adamw8bit).  Prints per-step wall span
(first kernel start → last kernel end), summed kernel time, idle fraction, kernel count, and
the top kernels of the steady-state steps.
    python scripts/step_timeline.py gpurun_out/prof_x/run_kernel_trace.csv [--marker adamw8bit]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--skip", type=int, default=1, help="steps to skip at the start")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    ends = [i for i, k in enumerate(ks) if re.search(a.marker, k[2])]
    steps = []
    for j in range(1, len(ends)):
        steps.append(ks[ends[j - 1] + 1: ends[j] + 1])
    steps = steps[a.skip:]
    agg = collections.Counter()
    cnt = collections.Counter()
    for i, st in enumerate(steps):
        wall = st[-1][1] - st[0][0]
        busy = 0
        last_end = st[0][0]
        for s, e, n in st:                      # union of intervals (kernels may overlap across streams)
            if e > last_end:
                busy += e - max(s, last_end)
                last_end = e
            agg[re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "anon"))[:80]] += e - s
            cnt[re.sub(r"\(.*", "", n.replace("(anonymous namespace)", "anon"))[:80]] += 1
        print(f"step {i}: wall {wall / 1e6:8.2f} ms  gpu-busy {busy / 1e6:8.2f} ms  idle {100 * (1 - busy / wall):5.1f}%  "
              f"kernels {len(st)}")
    n = max(1, len(steps))
    if steps:                                   # where the GPU waits for the host: largest gaps
        st = steps[-1]
        gaps = []
        for j in range(1, len(st)):
            g = st[j][0] - max(e for _, e, _ in st[:j]) if j < 400 else st[j][0] - st[j - 1][1]
            if g > 0:
                gaps.append((g, j))
        short = lambda nm: re.sub(r"\(.*", "", nm.replace("(anonymous namespace)", "anon"))[:60]   # noqa: E731
        print(f"\nlargest idle gaps of the last step (total {sum(g for g, _ in gaps) / 1e6:.2f} ms):")
        for g, j in sorted(gaps, reverse=True)[:12]:
            print(f"  {g / 1e3:8.1f} us  at kernel #{j:5d}  after {short(st[j - 1][2])}  before {short(st[j][2])}")
    print(f"\ntop kernels (ms/step over {n} steps):")
    for k, v in agg.most_common(a.top):
        print(f"  {v / 1e6 / n:8.3f} ms  x{cnt[k] / n:6.1f}  {k}")


if __name__ == "__main__":
    main()
