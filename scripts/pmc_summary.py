#!/usr/bin/env python3
"""Aggregate a rocprofv3 --pmc CSV per kernel: mean of each counter over dispatches.

    python scripts/pmc_summary.py gpurun_out/pmc_x/pmc_counter_collection.csv [--filter gemm]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"\(.*", "", name)
    return name[-70:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--filter", default="")
    ap.add_argument("--raw", action="store_true", help="also print every counter's mean per dispatch")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if a.filter and not re.search(a.filter, r["Kernel_Name"]):
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"], r["Grid_Size"], r["Workgroup_Size"])
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        v, ag, lds, grid, wg = meta[k]
        waves = int(grid) / 64
        line = [f"{k}", f"vgpr={v} agpr={ag} lds={lds} grid={grid} wg={wg} n={len(next(iter(cs.values())))}"]
        if "SQ_INSTS_VALU" in m:
            line.append(f"valu/wave={m['SQ_INSTS_VALU'] / waves:.0f}")
        if "SQ_INSTS_LDS" in m:
            line.append(f"lds/wave={m['SQ_INSTS_LDS'] / waves:.0f}")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_INSTS_LDS"):
            line.append(f"bankconf_cyc={m['SQ_LDS_BANK_CONFLICT']:.3g}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
            line.append(f"mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES']:.3g} busy={m['SQ_BUSY_CYCLES']:.3g}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if c in m:
                    line.append(f"{c[3:].lower()}/wave_cyc={m[c] / m['SQ_WAVE_CYCLES']:.3f}")
        print(" | ".join(line))
        if a.raw:
            print("    " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))


if __name__ == "__main__":
    main()
