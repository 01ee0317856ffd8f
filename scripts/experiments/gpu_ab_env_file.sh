#!/bin/bash
# Same-box A/B of one Python source file: alternates bench runs with $1 (old copy) swapped in for $2.
# usage: scripts/experiments/gpu_ab_env_file.sh <old_copy> <tracked_file>
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cp "$2" gpurun_out/new_copy.py
for rep in 1 2 3; do
for v in old new; do
if [ $v = old ]; then cp "$1" "$2"; else cp gpurun_out/new_copy.py "$2"; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_$v.log 2>&1 || exit 1
echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log)"
done
done
cp gpurun_out/new_copy.py "$2"
bash scripts/gpu_prof.sh v14
