#!/bin/bash
# run a subset of GPU tests: scripts/gpu_tests.sh <pytest -k expr or file>...
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest "$@" -q -x > gpurun_out/sub_tests.log 2>&1; rc=$?
tail -30 gpurun_out/sub_tests.log
exit $rc
