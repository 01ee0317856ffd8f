#!/bin/bash
# PMC passes for the g1w experiment (each pass its own run, --pmc only)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_g1w
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
D=$R/scripts/experiments/g1w/pmc_driver.py
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- python3 $D > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/sq2 -o pmc -- python3 $D > $OUT/sq2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/ta -o pmc -- python3 $D > $OUT/ta.log 2>&1 || exit 1
for d in sq sq2 ta; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py --raw $f > $OUT/$d.summary.txt; cat $OUT/$d.summary.txt; done
