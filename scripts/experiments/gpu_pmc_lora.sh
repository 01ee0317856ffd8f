#!/bin/bash
# LoRA kernel microbench + PMC passes (own runs, --pmc only) on the pair kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_lora
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 120 python3 $R/scripts/bench_lora.py > $OUT/bench.jsonl 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
export LORA_CASES=pair,proj_fwd,acc_dA_dx_drop
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/bench_lora.py > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/tcc -o pmc -- \
  python3 $R/scripts/bench_lora.py > $OUT/tcc.log 2>&1 || exit 1
for d in sq tcc; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f --filter lora > $OUT/$d.summary.txt; cat $OUT/$d.summary.txt; done
cat $OUT/bench.jsonl
