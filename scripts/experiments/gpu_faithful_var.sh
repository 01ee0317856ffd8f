#!/bin/bash
# run-to-run variance of the faithful #3 config: which hipBLASLt candidates each run picks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 LIPA_LT_VERBOSE=1
mkdir -p $R/gpurun_out/fvar
for i in 1 2 3 4; do
timeout -k 10 500 python bench.py --steps 10 --warmup 5 --grad-ckpt --ga-fusion 0 > $R/gpurun_out/fvar/$i.json 2>$R/gpurun_out/fvar/$i.err || { tail -5 $R/gpurun_out/fvar/$i.err; exit 1; }
echo "run $i $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/fvar/$i.json)"
grep "^\[lt\]" $R/gpurun_out/fvar/$i.err | sort | md5sum
done
