#!/bin/bash
# headline step (+ the faithful sub-record): LIPA_GEMM hybrid (default: gemm4w for the LoRA-fused projections
# and inside checkpointed layers, hipBLASLt for the other plain GEMMs) vs native (gemm4w everywhere) vs lt
# (hipBLASLt everywhere), interleaved on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/gemm_mode; mkdir -p $O
cd $R
for i in ${ITERS:-1 2 3}; do
  for g in ${MODES:-hybrid native lt}; do
    timeout -k 10 300 env LIPA_GEMM=$g python bench.py --faithful-steps ${FS:-0} --steps 10 --warmup 3 > $O/$g$i.json 2> $O/$g$i.err || { tail -5 $O/$g$i.err; exit 1; }
    echo "$g $i $(grep -o '"ms_per_step": [0-9.]*' $O/$g$i.json | tr '\n' ' ') $(grep -o '"peak_hbm_gib": [0-9.]*' $O/$g$i.json | head -1)"
  done
done
