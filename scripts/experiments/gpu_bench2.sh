#!/bin/bash
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for f in 1 0; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --ga-fusion $f > gpurun_out/bench_ga$f.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/bench_ga$f.log | tail -2 | cut -c1-300
done
bash scripts/gpu_prof.sh ga1 --ga-fusion 1
