#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_tests.log
case $rc in 0) ;; *) echo "tests rc=$rc"; exit $rc;; esac
timeout -k 10 300 python scripts/bench_gemm.py --m 2048 1024 --iters 20 --quick > gpurun_out/gemm_ab.log 2>&1 || exit $?
grep -E "TOTAL" gpurun_out/gemm_ab.log
