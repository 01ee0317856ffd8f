#!/bin/bash
# LoRA q+v projection on a side stream (LIPA_LORA_SIDE=1) vs in-stream: trainer tests under the side
# stream, probe (slab-sum kernel), full-step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/side
LIPA_LORA_SIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer_gpu.py tests/test_kernels_gpu.py -k "lora or trainer or ckpt" > $R/gpurun_out/side/tests.log 2>&1 || { tail -30 $R/gpurun_out/side/tests.log; exit 1; }
tail -1 $R/gpurun_out/side/tests.log
timeout -k 10 120 python3 scripts/experiments/lora_fwd_probe.py 2>/dev/null || exit 1
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_LORA_SIDE=1" "LIPA_LORA_SIDE=0"
