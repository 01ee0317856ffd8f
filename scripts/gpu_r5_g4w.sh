#!/bin/bash
# gemm4w change check: the gemm4w GPU tests, then the per-role GEMM A/B (gemm4w vs hipBLASLt) and the tile sweep.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r5g4w; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${K:-gemm4w}" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_roles.py > $O/roles.txt 2>&1 || { tail -5 $O/roles.txt; exit 1; }
cat $O/roles.txt
