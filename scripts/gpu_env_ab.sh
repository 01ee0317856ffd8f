#!/bin/bash
# bench.py A/B over environment settings, alternating, ROUNDS rounds (default 2).
# usage: BENCH_ARGS="--steps 10 --warmup 3" scripts/gpu_env_ab.sh <tag> "VAR=a" "VAR=b" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=$1; shift
OUT=$R/gpurun_out/envab_$TAG
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in "$@"; do
    env $e timeout -k 10 300 python3 $R/bench.py ${BENCH_ARGS:-} > $OUT/one.json 2> $OUT/one.err || { echo "[$e] failed"; tail -20 $OUT/one.err; exit 1; }
    echo "round $r [$e] $(grep -o '"ms_per_step": [0-9.]*' $OUT/one.json | head -1) $(grep -o '"faithful": {[^}]*' $OUT/one.json | grep -o '"ms_per_step": [0-9.]*' | head -1)" | tee -a $OUT/ab.txt
  done
done
