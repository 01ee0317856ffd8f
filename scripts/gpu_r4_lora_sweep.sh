#!/bin/bash
# LoRA / attention GPU tests, the LoRA-epilogue step A/B, then the gemm4w tile sweep.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_trainer_gpu.py $R/tests/test_kernels_gpu.py -k "lora or attention or attn or trainer or ckpt" > $R/gpurun_out/t_quad.txt 2>&1
rc=$?; tail -3 $R/gpurun_out/t_quad.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--steps 10 --warmup 3" bash $R/scripts/gpu_env_ab.sh epi "LIPA_LORA_EPI=1" "LIPA_LORA_EPI=0" || exit 1
timeout -k 10 400 python -u $R/scripts/sweep_gemm4w.py > $R/gpurun_out/sweep.txt 2>&1; rc=$?; cat $R/gpurun_out/sweep.txt; exit $rc
