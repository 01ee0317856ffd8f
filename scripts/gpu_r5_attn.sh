#!/bin/bash
# attention: numerics tests, then fwd/bwd timing (ours vs torch SDPA) at the bench shape and two long ones
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/attn_r5${1:+_$1}
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "attention or attn" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for sh in "--B 4 --S 512" "--B 2 --S 512" "--B 1 --S 2048" "--B 1 --S 8192"; do
  echo "$sh $(timeout -k 10 120 python -u $R/scripts/bench_attn.py $sh)" | tee -a $OUT/bench.txt || exit 1
done
