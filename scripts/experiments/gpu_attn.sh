#!/bin/bash
# attention numerics + microbenchmark + short bench.  usage: scripts/experiments/gpu_attn.sh
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
timeout -k 10 120 python scripts/bench_attn.py > gpurun_out/attn_bench.log 2>&1 || { tail -20 gpurun_out/attn_bench.log; exit 1; }
cat gpurun_out/attn_bench.log
timeout -k 10 120 python scripts/bench_attn.py --S 2048 --B 1 >> gpurun_out/attn_bench.log 2>&1 && tail -1 gpurun_out/attn_bench.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?
tail -2 gpurun_out/bench.log
exit $rc
