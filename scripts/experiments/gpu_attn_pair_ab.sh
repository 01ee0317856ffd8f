#!/bin/bash
# causal forward with paired query blocks (LIPA_ATTN_PAIR=1: heavy + light block per workgroup), QT 1 / 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/pair
for cfg in "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=2" "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=1"; do
env $cfg timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $R/gpurun_out/pair/tests.log 2>&1 || { echo "$cfg"; tail -30 $R/gpurun_out/pair/tests.log; exit 1; }
echo "$cfg: $(tail -1 $R/gpurun_out/pair/tests.log)"
done
for rep in 1 2; do for cfg in "LIPA_ATTN_PAIR=0 LIPA_ATTN_QT=2" "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=2" "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=1"; do
echo "[$cfg]"; for a in "" "--B 1 --S 2048" "--B 1 --S 8192" "--B 16 --S 512"; do env $cfg timeout -k 10 120 python3 scripts/bench_attn.py $a 2>/dev/null || exit 1; done; done; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_ATTN_PAIR=0 LIPA_ATTN_QT=2" "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=2" "LIPA_ATTN_PAIR=1 LIPA_ATTN_QT=1"
