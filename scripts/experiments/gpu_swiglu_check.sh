#!/bin/bash
# SwiGLU kernels on the (row, column-chunk) grid: numerics tests, bench, in-step kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=$R/gpurun_out/swiglu; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swiglu or gelu" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 > $OUT/kt.log 2>&1 || exit 1
python3 $R/scripts/step_timeline.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) --marker adamw8bit > $OUT/timeline.txt
rm -rf $OUT/kt
grep -E "step [01]|swiglu|rmsnorm|qk_norm|lora" $OUT/timeline.txt
