#!/bin/bash
# round-4 checks: gemm4w + trainer/ckpt GPU tests, then the bench A/B given as args.  usage: scripts/gpu_r4_check.sh <tag> [bench arg sets...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=$1; shift
OUT=$R/gpurun_out/chk_$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "gemm4w" \
   $R/tests/test_trainer_gpu.py > $OUT/tests.txt 2>&1
rc=$?; tail -6 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] && bash $R/scripts/gpu_bench_ab.sh $TAG "$@"
exit 0
