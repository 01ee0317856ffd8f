#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_decode_gpu.py tests/test_serving_gpu.py tests/test_moe.py -q -m gpu -x > $R/gpurun_out/dec_tests.log 2>&1; rc=$?
tail -5 $R/gpurun_out/dec_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/experiments/gpu_decode_prof.sh
