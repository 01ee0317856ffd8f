#!/bin/bash
# deferred running max in the attention forward (LIPA_ATTN_DEFER=8, cdna guide T13) vs exact (0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/defer
LIPA_ATTN_DEFER=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $R/gpurun_out/defer/tests.log 2>&1 || { tail -30 $R/gpurun_out/defer/tests.log; exit 1; }
tail -1 $R/gpurun_out/defer/tests.log
for rep in 1 2; do for d in 8 0; do echo "[defer=$d]"; for a in "" "--B 1 --S 2048" "--B 1 --S 8192"; do LIPA_ATTN_DEFER=$d timeout -k 10 120 python3 scripts/bench_attn.py $a 2>/dev/null || exit 1; done; done; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_ATTN_DEFER=8" "LIPA_ATTN_DEFER=0"
