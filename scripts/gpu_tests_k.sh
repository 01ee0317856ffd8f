#!/bin/bash
# run a pytest -k subset of the GPU tests: scripts/gpu_tests_k.sh "<-k expr>" [files...]
set -u
mkdir -p gpurun_out
K=$1; shift
FILES=${@:-tests}
timeout -k 10 600 python -u -m pytest $FILES -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/sub_tests.log 2>&1; rc=$?
tail -30 gpurun_out/sub_tests.log
exit $rc
