#!/bin/bash
# rocprofv3 kernel trace + stats of an arbitrary python command.  usage: scripts/gpu_prof_cmd.sh <tag> <script.py> [args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
S=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/$S "$@" > $OUT/log.txt 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 $OUT/log.txt
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -25 "$f" | cut -d, -f1-6
exit $rc
