#!/bin/bash
# Record of the BASELINE #2 A/B that fixed the rows per workgroup of the multi-adapter dB/dA launch (1 / 2 / 4
# 32-row steps per wave, interleaved): the switch it used is gone (lora.hip: 2 for rank 16 at >= 16 row blocks),
# so this now re-measures the shipped rule and its kernel trace.  Results: profiles/r4/lora_multi_adapter.txt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/lora_multi_ab; mkdir -p $O
cd $R
A="--mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4"
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.json) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json)"; }
run cfg2 python $R/bench.py --faithful-steps 0 --steps 6 --warmup 2 $A || exit 1
MARKER=adamw_k bash $R/scripts/gpu_step_prof.sh cfg2_multi $A > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -E "step 2|lora" $R/gpurun_out/prof_cfg2_multi/timeline.txt | grep -v " us  at" | head -12
