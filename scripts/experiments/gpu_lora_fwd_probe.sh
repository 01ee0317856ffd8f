#!/bin/bash
# lora_proj2 probe (timings hot / cold L2) + one SQ PMC pass on it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lora_fwd
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 120 python3 $R/scripts/experiments/lora_fwd_probe.py > $OUT/probe.jsonl 2>&1 || { cat $OUT/probe.jsonl; exit 1; }
cat $OUT/probe.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/experiments/lora_fwd_probe.py > $OUT/sq.log 2>&1 || exit 1
f=$(find $OUT/sq -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f --filter lora > $OUT/sq.summary.txt; cat $OUT/sq.summary.txt
