#!/bin/bash
# Decode step timing at serving batch sizes + kernel profile of a c=256 serving run (Qwen3-8B bf16).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_serve
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 $R/scripts/bench_decode.py --model qwen3-8b --batches 8 64 128 256 --ctx 512 --max-len 1024 \
  > $R/gpurun_out/decode_big.log 2>&1 || { tail -20 $R/gpurun_out/decode_big.log; exit 1; }
grep batch $R/gpurun_out/decode_big.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_serve -o run -- \
  python3 $R/scripts/bench_serve.py --inprocess random:qwen3-8b --dataset short --num-prompts 256 \
  --max-tokens 256 --concurrency 256 --max-batch 256 --max-model-len 1024 \
  > $R/gpurun_out/prof_serve/bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_serve/bench.log; exit 1; }
grep output_tok $R/gpurun_out/prof_serve/bench.log
S=$(find $R/gpurun_out/prof_serve -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py $S 1 30 > $R/gpurun_out/prof_serve/summary.txt
find $R/gpurun_out/prof_serve -name "*.csv" ! -name "*kernel_stats.csv" -delete; head -32 $R/gpurun_out/prof_serve/summary.txt
