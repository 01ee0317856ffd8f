#!/usr/bin/env python3
"""Summarise the innermost loop of each kernel in a hipcc -save-temps .s file.
usage: isa_loop.py file.s [name-substring]"""
import re, sys
src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2] if len(sys.argv) > 2 else ""
kern = None
done = set()
for i, l in enumerate(src):
    m = re.match(r"^(_Z\S+):", l)
    if m:
        kern = m.group(1)
    if "Loop Header" in l and kern and pat in kern and kern not in done:
        label = l.split(":")[0].strip()
        last = None
        for k in range(i + 1, min(len(src), i + 20000)):
            if re.match(r"^(_Z\S+):", src[k]):
                break
            if src[k].strip().startswith(("s_cbranch", "s_branch")) and src[k].strip().endswith(label):
                last = k
        if last is None:
            continue
        body = [x.strip() for x in src[i:last + 1] if x.strip() and not x.strip().startswith(";")]
        cnt = lambda p: sum(1 for x in body if re.match(p, x))
        print(f"{kern[:60]}: lines={len(body)} mfma={cnt(r'v_mfma')} valu={cnt(r'v_')} ds_read={cnt(r'ds_read')} "
              f"ds_write={cnt(r'ds_write')} vmem={cnt(r'(global|buffer)_')} waitcnt={cnt(r's_waitcnt')} "
              f"barrier={cnt(r's_barrier')} branches={cnt(r's_c?branch')}")
        done.add(kern)
