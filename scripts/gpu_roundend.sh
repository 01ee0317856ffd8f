#!/bin/bash
# Rehearsal of the driver's round-end GPU tiers: full `pytest -m gpu`, smoke(), 1-GPU bench.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1 || { tail -40 gpurun_out/gpu_tests_full.log; exit 1; }
tail -3 gpurun_out/gpu_tests_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1 || { tail -20 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log
