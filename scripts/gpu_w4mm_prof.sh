#!/bin/bash
# per-kernel times of the W4A16 microbench at the given row counts (rocprofv3 kernel trace --stats).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/w4prof_$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/scripts/bench_w4.py "$@" > $OUT/log.txt 2>&1
rc=$?
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
find $OUT -name "*kernel_trace.csv" -delete
exit $rc
