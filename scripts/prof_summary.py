#!/usr/bin/env python3
"""Top kernels from a rocprofv3 kernel_stats.csv (optionally per-step given --steps)."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total GPU time {tot/1e6:.1f} ms  ({tot/1e6/steps:.1f} ms per step over {steps:g})")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.2f} ms/step {float(r['Percentage']):6.2f}%  calls/step={int(r['Calls'])/steps:7.1f}"
          f"  avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:95]}")
