#!/bin/bash
# NF4 expansion with streaming stores (variants 4: 8 vectors/lane, 5: 4 vectors/lane) vs variant 3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python3 scripts/bench_dequant.py 2>/dev/null || exit 1
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_DEQUANT_VARIANT=3" "LIPA_DEQUANT_VARIANT=4" "LIPA_DEQUANT_VARIANT=5"
