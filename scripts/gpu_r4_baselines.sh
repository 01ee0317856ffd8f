#!/bin/bash
# BASELINE configs re-measured on the round-4 build (one box): #2 Qwen3-8B LoRA bf16 r16 q,k,v,o (ckpt and
# tuned), #4 Qwen3-14B QLoRA under the ZeRO-3 engine at world 1, replicated and partitioned NF4 bases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/cfg_r4; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 500 python $R/bench.py --faithful-steps 0 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.json) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json) $(grep -o '"peak_hbm_gib": [0-9.]*' $O/$tag.json | head -1)"; }
run cfg2_tuned --steps 6 --warmup 2 --mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 \
  --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 &&
run cfg2_ckpt --steps 6 --warmup 2 --mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 \
  --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 --grad-ckpt &&
run cfg4_zero3_w1 --steps 5 --warmup 2 --model qwen3-14b --strategy zero3 &&
run cfg4_zero3_w1_nf4part --steps 5 --warmup 2 --model qwen3-14b --strategy zero3 --ds-config $R/configs/ds_zero3_nf4_partition.json
