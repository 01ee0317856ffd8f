#!/bin/bash
# reference-faithful QLoRA config (gradient checkpointing on, sequential GA micro-steps of M = 1024):
# every NF4 weight is used 3x per micro-step (fwd, recompute, dX) -> fused register-dequant GEMM vs expand+hipBLASLt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/ckptf
i=0
for rep in 1 2; do for m in dequant fused; do
i=$((i+1))
LIPA_NF4_GEMM=$m timeout -k 10 400 python3 bench.py --steps 6 --warmup 2 --grad-ckpt --ga-fusion 0 > $R/gpurun_out/ckptf/$i.log 2>&1 || { tail -20 $R/gpurun_out/ckptf/$i.log; exit 1; }
echo "[ckpt faithful, LIPA_NF4_GEMM=$m] $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/ckptf/$i.log)"
done; done
