#!/bin/bash
# w4mm (W4A16 decode GEMM) numerics + microbench.  usage: scripts/gpu_w4mm.sh <tag> [M list]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=$1; shift
OUT=$R/gpurun_out/w4mm_$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py::test_w4mm_matches_fp32 $R/tests/test_quant_gpu.py > $OUT/tests.txt 2>&1
rc=$?; tail -4 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u $R/scripts/bench_w4.py "$@" > $OUT/bench.txt 2>&1
rc=$?; tail -3 $OUT/bench.txt; exit $rc
