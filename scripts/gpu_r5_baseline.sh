#!/bin/bash
# Round-5 baseline on one box: isolated per-role GEMM A/B (gemm4w vs hipBLASLt), then kernel traces of the
# headline step under LIPA_GEMM=native and =hybrid (per-kernel ms/step, idle gaps).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/r5base; mkdir -p $O
cd $R
timeout -k 10 300 python -u scripts/bench_roles.py > $O/roles.txt 2>&1 || { tail -5 $O/roles.txt; exit 1; }
cat $O/roles.txt
LIPA_GEMM=native bash scripts/gpu_step_prof.sh r5native || exit 1
LIPA_GEMM=hybrid bash scripts/gpu_step_prof.sh r5hybrid || exit 1
