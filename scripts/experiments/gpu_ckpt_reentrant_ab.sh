#!/bin/bash
# reentrant activation checkpointing (LIPA_CKPT_REENTRANT=1: no saved-tensor pack hooks in the first forward)
# vs non-reentrant on the host-bound reference-faithful #3 config
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p $R/gpurun_out/reent
LIPA_CKPT_REENTRANT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trainer_gpu.py > $R/gpurun_out/reent/tests.log 2>&1 || { tail -30 $R/gpurun_out/reent/tests.log; exit 1; }
tail -1 $R/gpurun_out/reent/tests.log
for rep in 1 2 3; do for v in 1 0; do
LIPA_CKPT_REENTRANT=$v timeout -k 10 500 python bench.py --steps 10 --warmup 4 --grad-ckpt --ga-fusion 0 > /tmp/r.json 2>/tmp/r.err || { tail -5 /tmp/r.err; exit 1; }
echo "[faithful #3, LIPA_CKPT_REENTRANT=$v] $(grep -o '"ms_per_step": [0-9.]*' /tmp/r.json) $(grep -o 'loss=[0-9.]*' /tmp/r.err | tail -1)"
done; done
