#!/bin/bash
# W4A16 decode GEMM microbench + BASELINE #5 AWQ merged-adapter inference bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 100 python scripts/experiments/dbg_w4.py > gpurun_out/dbg_w4.log 2>&1 &&
timeout -k 10 300 python scripts/bench_w4.py > gpurun_out/bench_w4.jsonl 2> gpurun_out/bench_w4.err &&
timeout -k 10 600 python -m llm_in_practise_amd.bench.awq_infer --model qwen3-8b --method awq --serve-requests 256 \
  --out gpurun_out/cfg5_awq_v2.json > gpurun_out/cfg5_v2.log 2>&1
rc=$?
grep -c "deterministic \[True, True, True\]" gpurun_out/dbg_w4.log; tail -c 1500 gpurun_out/cfg5_v2.log
exit $rc
