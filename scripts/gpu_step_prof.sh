#!/bin/bash
# rocprofv3 kernel trace of a few headline bench steps + the per-step timeline.  usage: scripts/gpu_step_prof.sh <tag> [bench args...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 --faithful-steps 0 --selective-steps 0 "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 $OUT/bench.log
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 $R/scripts/step_timeline.py "$f" --marker "${MARKER:-adamw8bit}" --skip "${SKIP:-1}" > $OUT/timeline.txt && head -60 $OUT/timeline.txt
rm -f "$f"
exit $rc
