#!/bin/bash
# attention numerics + fwd/bwd timing at the bench / long shapes, forward query-block A/B (LIPA_ATTN_QT)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention or flash or sdpa" > gpurun_out/attn_tests.log 2>&1 &&
for qt in 1 2; do
  for shp in "--B 4 --S 512" "--B 1 --S 2048" "--B 1 --S 8192" "--B 16 --S 512"; do
    LIPA_ATTN_QT=$qt timeout -k 10 120 python scripts/bench_attn.py $shp | sed "s/^/qt$qt /" >> gpurun_out/attn_bench.jsonl || exit 1
  done
done
rc=$?
grep -E "passed|failed" gpurun_out/attn_tests.log; cut -c1-120 gpurun_out/attn_bench.jsonl
exit $rc
