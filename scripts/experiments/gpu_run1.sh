#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1; rc=$?
tail -5 gpurun_out/tests.log
case $rc in 124|134|137|139) echo "abort rc=$rc"; exit $rc;; esac
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
bash scripts/experiments/gpu_pmc_gemm.sh cur --m 2048 --iters 5
