#!/bin/bash
# PMC counters of the GEMM microbench (own run: --pmc only, no trace domains).
# usage: scripts/experiments/gpu_pmc_gemm.sh <tag> [bench_gemm args]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT -o pmc -- \
  python3 $R/scripts/bench_gemm.py "$@" > $OUT/bench.log 2>&1
rc=$?
echo "pmc rc=$rc"
tail -5 $OUT/bench.log
exit $rc
