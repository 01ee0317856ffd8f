#!/bin/bash
# LoRA branch kernels: GPU tests, then microbench of the matrix-core lora_acc vs the VALU kernel.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lora" > gpurun_out/lora_tests.log 2>&1 || { tail -30 gpurun_out/lora_tests.log; exit 1; }
tail -2 gpurun_out/lora_tests.log
for V in mfma valu; do
  echo "lora_acc=$V"
  if [ $V = valu ]; then export LIPA_LORA_ACC_VALU=1; fi
  timeout -k 10 120 python scripts/bench_lora.py > gpurun_out/lora_$V.log 2>&1 || { tail -20 gpurun_out/lora_$V.log; exit 1; }
  grep case gpurun_out/lora_$V.log
done
