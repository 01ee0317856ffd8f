#!/bin/bash
# decode step (bf16 Qwen3-8B, ctx 1024): timing per batch + per-kernel profile at batch 64
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_decode
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 $R/scripts/bench_decode.py --model qwen3-8b --batches 1 8 32 64 --ctx 1024 \
  > $R/gpurun_out/decode_bf16.log 2>&1 || { tail -20 $R/gpurun_out/decode_bf16.log; exit 1; }
grep batch $R/gpurun_out/decode_bf16.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_decode -o run -- \
  python3 $R/scripts/bench_decode.py --model qwen3-8b --batches 64 --ctx 1024 --no-graph --steps 10 \
  > $R/gpurun_out/prof_decode/bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_decode/bench.log; exit 1; }
S=$(find $R/gpurun_out/prof_decode -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py $S 13 > $R/gpurun_out/prof_decode/summary.txt
head -30 $R/gpurun_out/prof_decode/summary.txt
