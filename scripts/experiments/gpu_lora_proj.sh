#!/bin/bash
set -u; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lora" > gpurun_out/lora_tests.log 2>&1 || { tail -30 gpurun_out/lora_tests.log; exit 1; }
tail -1 gpurun_out/lora_tests.log
timeout -k 10 100 python scripts/bench_lora.py > gpurun_out/lora.log 2>&1 || exit 1; grep proj gpurun_out/lora.log
timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/bench_lp.log 2>&1 || exit 1
grep -o '[0-9.]* ms/step  [0-9,]* tok/s' gpurun_out/bench_lp.log
