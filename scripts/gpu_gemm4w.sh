#!/bin/bash
# gemm4w vs hipBLASLt at the step shapes.  usage: scripts/gpu_gemm4w.sh <tag>
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=.
TAG=${1:-g4w}
SPLITS=${SPLITS:-0,1,2} timeout -k 10 300 python -u scripts/bench_gemm4w.py > gpurun_out/${TAG}.txt 2>&1
rc=$?; cat gpurun_out/${TAG}.txt; exit $rc
