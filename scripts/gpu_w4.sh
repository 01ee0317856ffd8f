#!/bin/bash
# NF4-in-gemm4w: numerics tests, then the per-shape A/B.  usage: scripts/gpu_w4.sh <tag>
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=.
TAG=${1:-w4}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm4w_nf4 or gemm4w_asym or gemm4w_swiglu or nf4_dequant_fast" > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gemm4w_nf4.py > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; cat gpurun_out/${TAG}_ab.txt; exit $rc
