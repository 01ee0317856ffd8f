#!/bin/bash
# per-kernel profile of one Qwen3-8B bf16 decode step (eager, 10 steps) at batch 8 and 256, ctx 512
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for B in 8 256; do
  mkdir -p $R/gpurun_out/prof_dec$B
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dec$B -o run -- \
    python3 $R/scripts/bench_decode.py --model qwen3-8b --batches $B --ctx 512 --max-len 1024 --no-graph --steps 10 \
    > $R/gpurun_out/prof_dec$B/bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_dec$B/bench.log; exit 1; }
  S=$(find $R/gpurun_out/prof_dec$B -name "*kernel_stats.csv" | head -1)
  python3 $R/scripts/prof_summary.py $S 13 25 > $R/gpurun_out/prof_dec$B/summary.txt
  echo "== batch $B"; head -22 $R/gpurun_out/prof_dec$B/summary.txt
  find $R/gpurun_out/prof_dec$B -name "*.csv" ! -name "*kernel_stats.csv" -delete
done
