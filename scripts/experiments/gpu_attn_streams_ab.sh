#!/bin/bash
# attention backward: dK/dV on a side stream beside dQ (LIPA_ATTN_BWD_STREAMS=1, default) vs one stream
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/attn2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" tests/test_trainer_gpu.py > $R/gpurun_out/attn2/tests.log 2>&1 || { tail -30 $R/gpurun_out/attn2/tests.log; exit 1; }
tail -1 $R/gpurun_out/attn2/tests.log
for i in 1 0 1 0; do echo "streams=$i"; LIPA_ATTN_BWD_STREAMS=$i timeout -k 10 120 python3 scripts/bench_attn.py 2>/dev/null || exit 1; LIPA_ATTN_BWD_STREAMS=$i timeout -k 10 120 python3 scripts/bench_attn.py --B 1 --S 2048 2>/dev/null || exit 1; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_ATTN_BWD_STREAMS=1" "LIPA_ATTN_BWD_STREAMS=0"
