#!/bin/bash
# checkpointed BASELINE configs (#2 ckpt, #3 faithful) with the reentrant default, vs LIPA_CKPT_REENTRANT=0
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 1 0 1; do
LIPA_CKPT_REENTRANT=$v timeout -k 10 500 python bench.py --steps 6 --warmup 3 --mode lora --targets q_proj,k_proj,v_proj,o_proj --lora-r 16 --lora-alpha 32 \
  --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 --grad-ckpt > /tmp/c2.json 2>/tmp/c2.err || { tail -5 /tmp/c2.err; exit 1; }
echo "[#2 ckpt, reentrant=$v] $(grep -o '"value": [0-9.]*' /tmp/c2.json) $(grep -o '"ms_per_step": [0-9.]*' /tmp/c2.json)"
LIPA_CKPT_REENTRANT=$v timeout -k 10 500 python bench.py --steps 8 --warmup 3 --grad-ckpt --ga-fusion 0 > /tmp/c3.json 2>/tmp/c3.err || { tail -5 /tmp/c3.err; exit 1; }
echo "[#3 faithful, reentrant=$v] $(grep -o '"value": [0-9.]*' /tmp/c3.json) $(grep -o '"ms_per_step": [0-9.]*' /tmp/c3.json)"
done
