#!/bin/bash
# MFMA decode attention (fused KV append) + hipBLASLt dense path: tests, decode-step timing, serving vs reference
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_decode_gpu.py tests/test_serving_gpu.py \
  > gpurun_out/dec2_tests.log 2>&1 || { tail -40 gpurun_out/dec2_tests.log; exit 1; }
tail -2 gpurun_out/dec2_tests.log
timeout -k 10 300 python3 scripts/bench_decode.py --model qwen3-8b --batches 8 64 128 256 --ctx 512 --max-len 1024 \
  > gpurun_out/decode_big2.log 2>&1 || { tail -20 gpurun_out/decode_big2.log; exit 1; }
grep batch gpurun_out/decode_big2.log
bash scripts/experiments/gpu_serve_ref.sh
