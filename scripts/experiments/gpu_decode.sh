#!/bin/bash
# MoE kernel tests + decode-step microbenchmarks (eager vs hipGraph) on one MI355X
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_moe.py -q -m gpu > gpurun_out/moe_tests.log 2>&1; rc=$?
tail -3 gpurun_out/moe_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_skinny.py > gpurun_out/skinny.log 2>&1 || { tail -20 gpurun_out/skinny.log; exit 1; }
cat gpurun_out/skinny.log | grep shape
timeout -k 10 400 python scripts/bench_decode.py --model qwen3-8b --batches 1 8 32 64 --ctx 1024 \
  > gpurun_out/decode_bf16.log 2>&1 || { tail -20 gpurun_out/decode_bf16.log; exit 1; }
cat gpurun_out/decode_bf16.log | grep batch
timeout -k 10 400 python scripts/bench_decode.py --model qwen3-8b --nf4 --batches 1 8 32 64 --ctx 1024 \
  > gpurun_out/decode_nf4.log 2>&1 || { tail -20 gpurun_out/decode_nf4.log; exit 1; }
cat gpurun_out/decode_nf4.log | grep batch
