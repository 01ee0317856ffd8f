#!/bin/bash
# Serving throughput at the reference's published concurrency levels (vLLM on 1× RTX 3090,
# Qwen3-8B BF16, output len 256, ignore-eos): our engine + OpenAI server in-process, random-init weights.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 800 python scripts/bench_serve.py --spawn --inprocess random:qwen3-8b --dataset short --num-prompts 256 \
  --max-tokens 256 --concurrency 8 16 32 64 128 256 --max-batch 256 --max-model-len 1024 \
  --out gpurun_out/serve_ref.json > gpurun_out/serve_ref.log 2>&1; rc=$?
grep output_tok gpurun_out/serve_ref.log || tail -20 gpurun_out/serve_ref.log
exit $rc
