#!/bin/bash
# next-layer NF4 expansion by a small persistent grid on a side stream (LIPA_NF4_BG=G) vs inline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/nf4bg
LIPA_NF4_BG=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer_gpu.py > $R/gpurun_out/nf4bg/tests.log 2>&1 || { tail -30 $R/gpurun_out/nf4bg/tests.log; exit 1; }
tail -1 $R/gpurun_out/nf4bg/tests.log
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_NF4_BG=0" "LIPA_NF4_BG=64" "LIPA_NF4_BG=128" "LIPA_NF4_BG=256"
