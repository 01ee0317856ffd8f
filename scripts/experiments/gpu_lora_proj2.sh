#!/bin/bash
set -u; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for RW in 8 16 8 16; do echo "rw=$RW"
LIPA_LORA_PROJ_RW=$RW timeout -k 10 100 python scripts/bench_lora.py > gpurun_out/lora.log 2>&1 || exit 1; grep proj gpurun_out/lora.log
done
