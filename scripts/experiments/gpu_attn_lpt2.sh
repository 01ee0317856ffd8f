#!/bin/bash
# longest-first causal grid with runs of exactly one XCD's share (fix of the 2-XCD runs at QT = 2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/lpt2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > $R/gpurun_out/lpt2/tests.log 2>&1 || { tail -30 $R/gpurun_out/lpt2/tests.log; exit 1; }
tail -1 $R/gpurun_out/lpt2/tests.log
for i in 1 2 1 2; do echo "qt=$i"; for a in "" "--B 1 --S 2048" "--B 1 --S 8192" "--B 16 --S 512"; do LIPA_ATTN_QT=$i timeout -k 10 120 python3 scripts/bench_attn.py $a 2>/dev/null || exit 1; done; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_ATTN_QT=2" "LIPA_ATTN_QT=1"
