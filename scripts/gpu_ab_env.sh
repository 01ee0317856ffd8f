#!/bin/bash
# Same-box A/B of environment settings on the full bench: scripts/gpu_ab_env.sh "A=1" "A=2 B=3" ...
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
i=0
for rep in 1 2; do
for cfg in "$@"; do
i=$((i+1))
env $cfg timeout -k 10 300 python bench.py --steps ${AB_STEPS:-20} --warmup 3 > gpurun_out/abenv_$i.log 2>&1 || { tail -20 gpurun_out/abenv_$i.log; exit 1; }
echo "[$cfg] $(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' gpurun_out/abenv_$i.log) $(grep -o 'max_mem[^,]*' gpurun_out/abenv_$i.log)"
done
done
