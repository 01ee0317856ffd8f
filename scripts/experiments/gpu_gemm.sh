#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_tests.log
case $rc in 124|134|137|139) echo "abort rc=$rc"; exit $rc;; esac
for mt in 8 16; do
  LIPA_GEMM_MT=$mt timeout -k 10 300 python scripts/bench_gemm.py --iters 20 > gpurun_out/gemm_mt$mt.log 2>&1 || exit $?
  grep -E "TOTAL|nf4" gpurun_out/gemm_mt$mt.log | head -40
done
