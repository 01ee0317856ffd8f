#!/bin/bash
# BASELINE #4 (Qwen3-14B QLoRA, ZeRO-3 engine, world 1): step timeline + top kernels, and the same model
# through the DDP path for the ZeRO-3 overhead
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/z3prof; mkdir -p $OUT
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 bench.py --model qwen3-14b --steps 6 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/ddp 14b /' || exit 1
timeout -k 10 400 python3 bench.py --model qwen3-14b --strategy zero3 --steps 6 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed 's/^/zero3 14b /' || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- \
  python3 $R/bench.py --model qwen3-14b --strategy zero3 --steps 3 --warmup 2 > $OUT/kt.log 2>&1 || exit 1
python3 $R/scripts/step_timeline.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) --marker "adamw|sumsq" --top 25 > $OUT/timeline.txt
rm -rf $OUT/kt
head -45 $OUT/timeline.txt
