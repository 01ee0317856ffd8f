#!/bin/bash
# hipBLASLt workspace size (LIPA_LT_WS_MB) x gate|up dX K-slices (LIPA_DX_SPLIT): a larger workspace admits
# the library's own split-K / stream-K reductions for the unsplit GEMM
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 LIPA_LT_VERBOSE=1
mkdir -p $R/gpurun_out/ltws
i=0
for rep in 1 2; do for cfg in "LIPA_LT_WS_MB=64" "LIPA_LT_WS_MB=512" "LIPA_LT_WS_MB=512 LIPA_DX_SPLIT=1 LIPA_LT_CANDIDATES=16"; do
i=$((i+1))
env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 4 > $R/gpurun_out/ltws/$i.json 2>$R/gpurun_out/ltws/$i.err || { tail -5 $R/gpurun_out/ltws/$i.err; exit 1; }
echo "[$cfg] $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/ltws/$i.json)"
grep "^\[lt\]" $R/gpurun_out/ltws/$i.err | grep "n=2048 k=24576\|k=24576\|m=4096 n=2048 k=12288 b=\|b=2" | head -3
done; done
