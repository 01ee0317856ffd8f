#!/bin/bash
# reference-faithful #3 (ckpt on, sequential GA): longer warmup, and with the round-2-late kernels switched off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "LIPA_PROJ2_IMPL=1" "LIPA_PROJ2_IMPL=0 LIPA_LORA_DX_RPT=4 LIPA_ATTN_LPT=2" "LIPA_PROJ2_IMPL=1"; do
env $cfg timeout -k 10 500 python bench.py --steps 10 --warmup 5 --grad-ckpt --ga-fusion 0 > /tmp/f.json 2>/tmp/f.err || { tail -5 /tmp/f.err; exit 1; }
echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' /tmp/f.json)"
done
