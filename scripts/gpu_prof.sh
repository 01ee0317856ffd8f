#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run.  usage: scripts/gpu_prof.sh <tag> [bench args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 $OUT/bench.log
find $OUT -name "*kernel_stats.csv" | head -3
