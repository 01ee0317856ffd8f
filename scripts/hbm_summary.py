#!/usr/bin/env python3
"""Per-kernel HBM traffic of the bench step: rocprofv3 FETCH_SIZE / WRITE_SIZE passes (KB per dispatch,
mean over dispatches) joined with the kernel-trace durations of an unperturbed run (mean µs), giving the
achieved DRAM-side bandwidth per kernel.  FETCH_SIZE / WRITE_SIZE count TCC (L2) traffic to and from
memory (MALL/HBM), so an L2-resident operand does not appear in them.

    python scripts/hbm_summary.py <kernel_trace.csv> <fetch_pmc.csv> <write_pmc.csv> [--top 25]
"""
import argparse
import collections
import csv
import re


def short(n):
    n = n.replace("(anonymous namespace)", "anon")
    return re.sub(r"\(.*", "", n)[:72]


def pmc_means(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    dur, cnt = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(a.trace)):
        k = short(r["Kernel_Name"])
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    fetch, write = pmc_means(a.fetch, "FETCH_SIZE"), pmc_means(a.write, "WRITE_SIZE")
    print(f"{'kernel':72s} {'calls':>6s} {'us/call':>8s} {'rd MB':>8s} {'wr MB':>8s} {'GB/s':>7s}")
    for k, tot in dur.most_common(a.top):
        us = tot / cnt[k]
        rd, wr = fetch.get(k, float("nan")) / 1024, write.get(k, float("nan")) / 1024
        print(f"{k:72s} {cnt[k]:6d} {us:8.1f} {rd:8.2f} {wr:8.2f} {(rd + wr) * 1e3 / us:7.0f}")


if __name__ == "__main__":
    main()
