#!/bin/bash
# BASELINE config #4 rehearsal on one GPU: Qwen3-14B QLoRA with the ZeRO-3 engine (ds_zero3_config.json)
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --model qwen3-14b --strategy zero3 --steps 5 --warmup 2 > gpurun_out/zero3_14b.log 2>&1 || { tail -30 gpurun_out/zero3_14b.log; exit 1; }
tail -2 gpurun_out/zero3_14b.log
timeout -k 10 400 python bench.py --model qwen3-14b --steps 5 --warmup 2 > gpurun_out/ddp_14b.log 2>&1 || { tail -30 gpurun_out/ddp_14b.log; exit 1; }
tail -2 gpurun_out/ddp_14b.log
