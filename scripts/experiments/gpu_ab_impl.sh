#!/bin/bash
# Same-box A/B of the NF4 GEMM generations: gemm tests, then alternating full-bench runs.
# usage: scripts/experiments/gpu_ab_impl.sh <impl> <impl> ...
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or nf4 or int4" --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -20 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
for rep in 1 2; do
for impl in "$@"; do
LIPA_GEMM_IMPL=$impl timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_$impl.log 2>&1 || exit 1
echo "impl=$impl $(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' gpurun_out/ab_$impl.log)"
done
done
