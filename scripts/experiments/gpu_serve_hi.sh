#!/bin/bash
# High-concurrency serving levels of the reference table (c=64/128/256, 256 prompts, 256 output tokens)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_serve.py --spawn --inprocess random:qwen3-8b --dataset short --num-prompts 256 \
  --max-tokens 256 --concurrency ${CONC:-64 128 256} --max-batch 256 --max-model-len 1024 ${EXTRA:-} \
  --out gpurun_out/serve_hi.json > gpurun_out/serve_hi.log 2>&1; rc=$?
grep output_tok gpurun_out/serve_hi.log || tail -20 gpurun_out/serve_hi.log
exit $rc
