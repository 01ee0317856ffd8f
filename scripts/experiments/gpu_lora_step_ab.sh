#!/bin/bash
# LoRA GPU tests, then alternating full-step bench: matrix-core lora_acc (default) vs the VALU kernel.
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lora" > gpurun_out/lora_tests.log 2>&1 || { tail -30 gpurun_out/lora_tests.log; exit 1; }
tail -1 gpurun_out/lora_tests.log
for rep in 1 2; do
for v in mfma valu; do
if [ $v = valu ]; then V=1; else V=; fi
env ${V:+LIPA_LORA_ACC_VALU=1} timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/ab_lora_$v.log 2>&1 || exit 1
echo "lora_acc=$v $(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' gpurun_out/ab_lora_$v.log)"
done
done
