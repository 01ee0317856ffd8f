#!/bin/bash
# BASELINE #5 end to end: merged-LoRA Qwen3-8B, bf16 vs int4 (RTN g128) decode per batch + prefill + quality.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/awq_$1; mkdir -p $OUT
timeout -k 10 900 python -u -m llm_in_practise_amd.bench.awq_infer --method ${METHOD:-rtn} --batches 1 2 8 16 32 64 256 \
  --ppl-prompts 2 --ppl-new 32 --out $OUT/awq.json > $OUT/log.txt 2>&1
rc=$?; tail -30 $OUT/log.txt; exit $rc
