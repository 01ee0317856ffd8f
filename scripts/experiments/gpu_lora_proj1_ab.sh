#!/bin/bash
# single-branch lora_proj through the split-K kernel (LIPA_PROJ2_IMPL=1) vs the 8/16-row kernel (0) on BASELINE #2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/proj1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_trainer_gpu.py -k "lora or trainer or ckpt" > $R/gpurun_out/proj1/tests.log 2>&1 || { tail -30 $R/gpurun_out/proj1/tests.log; exit 1; }
tail -1 $R/gpurun_out/proj1/tests.log
i=0
for rep in 1 2; do for impl in 1 0; do
i=$((i+1))
LIPA_PROJ2_IMPL=$impl timeout -k 10 400 python bench.py --steps 8 --warmup 3 --mode lora --targets q_proj,k_proj,v_proj,o_proj \
  --lora-r 16 --lora-alpha 32 --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 > $R/gpurun_out/proj1/$i.json 2>/dev/null || exit 1
echo "[#2 LoRA bf16 no-ckpt, LIPA_PROJ2_IMPL=$impl] $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/proj1/$i.json)"
done; done
