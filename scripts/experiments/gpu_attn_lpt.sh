#!/bin/bash
# attention longest-first grid order (LIPA_ATTN_LPT) : numerics, kernel timing at the bench / long shapes, full bench A/B
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention or flash" > gpurun_out/lpt_tests.log 2>&1 || { tail -20 gpurun_out/lpt_tests.log; exit 1; }
tail -1 gpurun_out/lpt_tests.log
for rep in 1 2; do for l in 1 0; do
  for shp in "--B 4 --S 512" "--B 1 --S 2048"; do
    LIPA_ATTN_LPT=$l timeout -k 10 120 python scripts/bench_attn.py $shp | sed "s/^/lpt$l /" | cut -c1-150 || exit 1
  done
done; done
bash scripts/gpu_ab_env.sh LIPA_ATTN_LPT=1 LIPA_ATTN_LPT=0
