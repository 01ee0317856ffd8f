#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_trainer_gpu.py -q -x -m gpu > gpurun_out/lora_tests.log 2>&1; rc=$?
tail -5 gpurun_out/lora_tests.log
case $rc in 0) ;; *) echo "tests rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_lora.log 2>&1 || exit $?
tail -2 gpurun_out/bench_lora.log
