#!/bin/bash
# step timeline (GPU busy vs wall) of the reference-faithful #3 config
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fprof; mkdir -p $OUT
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 --grad-ckpt --ga-fusion 0 > $OUT/kt.log 2>&1 || exit 1
python3 $R/scripts/step_timeline.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) --marker adamw8bit --top 12 > $OUT/timeline.txt
rm -rf $OUT/kt
head -30 $OUT/timeline.txt
