#!/bin/bash
# Multi-adapter LoRA kernels (lora_proj_m / lora_proj_cols / lora_acc_jobs / lora_dxc): GPU numerics, then
# BASELINE #2 (bf16 LoRA r16 on q,k,v,o) with the multi-adapter path vs the per-adapter kernels
# (LIPA_LORA_MULTI=0), interleaved on one box, and a kernel trace of the new #2 step.
# (The shared-x dA grouping A/B it also ran used a switch that is gone with the grouping: profiles/r4/lora_multi_adapter.txt.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/lora_multi; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lora_multi_gpu.py \
  "tests/test_trainer_gpu.py::test_lora_dx_as_gemm_c_matches_read_modify_write" \
  "tests/test_trainer_gpu.py::test_grad_ckpt_lora_dropout_same_gradients" \
  "tests/test_trainer_gpu.py::test_lora_pair_kernels_match_single_branch_path" > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4"
run() { local tag=$1; shift; timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $O/$tag.json) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.json)"; }
for i in 1 2; do
  run multi_$i LIPA_LORA_MULTI=1 python $R/bench.py --faithful-steps 0 --steps 6 --warmup 2 $A || exit 1
  run single_$i LIPA_LORA_MULTI=0 python $R/bench.py --faithful-steps 0 --steps 6 --warmup 2 $A || exit 1
done
run multi_ckpt LIPA_LORA_MULTI=1 python $R/bench.py --faithful-steps 0 --steps 6 --warmup 2 $A --grad-ckpt || exit 1
MARKER=adamw_k bash $R/scripts/gpu_step_prof.sh cfg2_multi $A > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -E "step 2|lora" $R/gpurun_out/prof_cfg2_multi/timeline.txt | head -20
