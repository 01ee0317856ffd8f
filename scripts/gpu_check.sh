#!/bin/bash
# One GPU session: tests -> smoke -> bench.  Stops at the first crash/timeout (never retries).
# usage: scripts/gpu_check.sh [pytest-args...]
set -u
OUT=gpurun_out
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/summary.log
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/summary.log
  tail -n 25 $OUT/$name.log
  if crashed $rc; then echo "ABORT after $name (rc=$rc)" | tee -a $OUT/summary.log; exit $rc; fi
  return 0
}
rocm-smi --showproductname > $OUT/gpu.txt 2>&1 || true
run smoke 300 python __graft_entry__.py smoke
run tests 900 python -m pytest tests -m gpu -q "$@"
run bench 600 python bench.py --steps ${BENCH_STEPS:-5} --warmup ${BENCH_WARMUP:-2}
