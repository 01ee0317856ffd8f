#!/bin/bash
# End-of-round-2 re-measure of BASELINE configs #2, #3 (faithful + tuned) and #4 (ZeRO-3, world 1) on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/cfg_r2; mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 500 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.json) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json)"; }
run cfg3_tuned --steps 10 --warmup 3 &&
run cfg3_faithful --steps 6 --warmup 2 --grad-ckpt --ga-fusion 0 &&
run cfg2_ckpt --steps 6 --warmup 2 --mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 \
  --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 --grad-ckpt &&
run cfg2_tuned --steps 6 --warmup 2 --mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 \
  --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 &&
run cfg4_zero3_w1 --steps 5 --warmup 2 --model qwen3-14b --strategy zero3
