#!/bin/bash
# BASELINE #5 (merged-LoRA Qwen3-8B, bf16 vs int4 RTN g128): awq_infer per decode batch + prefill, then a
# kernel-trace breakdown per batch (bf16 and int4 kernels in one stats table)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/awq_prof${1:+_$1}; mkdir -p $OUT
timeout -k 10 600 python -u -m llm_in_practise_amd.bench.awq_infer --method rtn --batches 1 8 32 64 256 \
  --ppl-prompts 1 --ppl-new 8 --out $OUT/awq.json > $OUT/log.txt 2>&1 || { tail -30 $OUT/log.txt; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/awq.json')); print('speedup', d['decode_speedup']); print('prefill bf16', d['bf16']['prefill']['ms'], 'int4', d['int4']['prefill']['ms'])"
cd /tmp && export TMPDIR=/tmp
for b in 64 256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$b -o kt -- python3 -m llm_in_practise_amd.bench.awq_infer --method rtn --batches $b --steps 10 --ppl-prompts 1 --ppl-new 4 > $OUT/kt_$b.log 2>&1 || exit 1
  echo "== batch $b"; python3 $R/scripts/prof_summary.py $(find $OUT/kt_$b -name "*kernel_stats.csv" | head -1) 1 25
done | tee $OUT/kt_summary.txt
