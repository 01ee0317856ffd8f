#!/bin/bash
# host-side profile of the reference-faithful #3 config (host-bound: 13-15 % GPU idle)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fcprof; mkdir -p $OUT
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -m cProfile -o $OUT/prof.out bench.py --steps 4 --warmup 2 --grad-ckpt --ga-fusion 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
python3 - <<PY > $OUT/top.txt
import pstats
p = pstats.Stats("$OUT/prof.out"); p.sort_stats("tottime").print_stats(45)
PY
python3 - <<PY > $OUT/cum.txt
import pstats
p = pstats.Stats("$OUT/prof.out"); p.sort_stats("cumulative").print_stats(60)
PY
rm -f $OUT/prof.out
grep -A50 "ncalls" $OUT/top.txt | cut -c1-200 | head -55
