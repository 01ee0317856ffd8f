#!/bin/bash
# NF4 GEMM numerics + A/B microbenchmark.  usage: scripts/experiments/gpu_gemm3.sh <impls...>
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or nf4 or int4" --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_tests.log
case $rc in 0) ;; *) echo "tests rc=$rc"; exit $rc;; esac
timeout -k 10 300 python scripts/bench_gemm.py --m 2048 --iters 20 --quick --impls "$@" > gpurun_out/gemm_ab.log 2>&1 || exit $?
cat gpurun_out/gemm_ab.log
