#!/bin/bash
# serving benchmark on one MI355X: our OpenAI server in-process, random-init weights, byte tokenizer
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=${1:-random:qwen3-8b}
timeout -k 10 900 python scripts/bench_serve.py --inprocess $MODEL --num-prompts 64 --max-tokens 128 \
  --concurrency 1 8 32 64 --out gpurun_out/serve_bench.json > gpurun_out/serve_bench.log 2>&1; rc=$?
tail -8 gpurun_out/serve_bench.log
exit $rc
