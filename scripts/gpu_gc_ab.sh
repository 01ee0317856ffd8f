#!/bin/bash
# faithful sub-record with Python's automatic GC (LIPA_GC_INTERVAL=0) vs manual GC (default), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/gc_ab; mkdir -p $O
cd $R
for i in 1 2 3 4; do
  for g in 0 100; do
    timeout -k 10 300 env LIPA_GC_INTERVAL=$g python bench.py --steps 10 --warmup 3 --faithful-steps 5 > $O/gc$g.$i.json 2> $O/gc$g.$i.err || { tail -5 $O/gc$g.$i.err; exit 1; }
    echo "gc_interval=$g $i $(grep -o '"ms_per_step": [0-9.]*' $O/gc$g.$i.json | tr '\n' ' ')"
  done
done
