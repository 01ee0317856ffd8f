#!/bin/bash
# int4 decode GEMM + custom all-reduce tests, W4A16 microbench, AWQ decode bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_custom_allreduce_gpu.py \
  tests/test_quant_gpu.py > gpurun_out/w4_car_tests.log 2>&1 &&
timeout -k 10 300 python scripts/bench_w4.py > gpurun_out/bench_w4.jsonl 2> gpurun_out/bench_w4.err &&
timeout -k 10 600 python -m llm_in_practise_amd.bench.awq_infer --model qwen3-8b --method awq --serve-requests 256 \
  --out gpurun_out/cfg5_awq_v2.json > gpurun_out/cfg5_v2.log 2>&1
rc=$?
tail -5 gpurun_out/w4_car_tests.log; cat gpurun_out/bench_w4.jsonl | cut -c1-220; tail -c 1200 gpurun_out/cfg5_v2.log
exit $rc
