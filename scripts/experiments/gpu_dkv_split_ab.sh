#!/bin/bash
# causal dK/dV: heavy key blocks split over two workgroups + fp32 finalize (LIPA_ATTN_DKV_SPLIT=1, default) vs whole blocks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/dkv
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" tests/test_trainer_gpu.py > $R/gpurun_out/dkv/tests.log 2>&1 || { tail -30 $R/gpurun_out/dkv/tests.log; exit 1; }
tail -1 $R/gpurun_out/dkv/tests.log
for i in 1 0 1 0; do echo "split=$i"; LIPA_ATTN_DKV_SPLIT=$i timeout -k 10 120 python3 scripts/bench_attn.py 2>/dev/null || exit 1; LIPA_ATTN_DKV_SPLIT=$i timeout -k 10 120 python3 scripts/bench_attn.py --B 1 --S 2048 2>/dev/null || exit 1; done
AB_STEPS=20 bash scripts/gpu_ab_env.sh "LIPA_ATTN_DKV_SPLIT=1" "LIPA_ATTN_DKV_SPLIT=0"
