#!/bin/bash
# kernel-trace stats + SQ PMC pass of the split-K lora_proj2 probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/proj2prof
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/scripts/experiments/lora_fwd_probe.py > $OUT/kt.log 2>&1 || exit 1
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); head -8 $f
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/experiments/lora_fwd_probe.py > $OUT/sq.log 2>&1 || exit 1
f=$(find $OUT/sq -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f --filter lora > $OUT/sq.summary.txt; cat $OUT/sq.summary.txt
