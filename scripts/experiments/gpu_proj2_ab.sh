#!/bin/bash
# split-K lora_proj2 (LIPA_PROJ2_IMPL=1, default) vs the 8-row kernel (0): tests, probe, full-step A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/proj2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora" tests/test_trainer_gpu.py > $R/gpurun_out/proj2/tests.log 2>&1 || { tail -30 $R/gpurun_out/proj2/tests.log; exit 1; }
tail -2 $R/gpurun_out/proj2/tests.log
for i in 1 0; do LIPA_PROJ2_IMPL=$i timeout -k 10 120 python3 scripts/experiments/lora_fwd_probe.py 2>/dev/null || exit 1; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_PROJ2_IMPL=1 LIPA_LORA_DX_RPT=16" "LIPA_PROJ2_IMPL=1 LIPA_LORA_DX_RPT=4" "LIPA_PROJ2_IMPL=0 LIPA_LORA_DX_RPT=4"
