#!/bin/bash
# bench.py A/B: alternating runs of the given arg sets.  usage: scripts/gpu_bench_ab.sh <tag> "<args A>" "<args B>" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; shift
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 $R/bench.py $a > $OUT/run$i.json 2> $OUT/run$i.err || { echo "run $i ($a) failed"; tail -20 $OUT/run$i.err; exit 1; }
  echo "[$a] $(grep -h '\[bench\]' $OUT/run$i.err | tail -2 | tr '\n' ' ')"
done
