#!/bin/bash
# headline step: number of hipBLASLt heuristic candidates timed in-step per shape (LIPA_LT_CANDIDATES), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/lt_cand; mkdir -p $O
cd $R
for i in 1 2; do
  for c in 4 8 16; do
    timeout -k 10 300 env LIPA_LT_CANDIDATES=$c python bench.py --faithful-steps 0 --steps 10 --warmup 4 > $O/c$c.$i.json 2> $O/c$c.$i.err || { tail -5 $O/c$c.$i.err; exit 1; }
    echo "candidates=$c $i $(grep -o '"ms_per_step": [0-9.]*' $O/c$c.$i.json)"
  done
done
