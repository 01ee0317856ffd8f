#!/bin/bash
# PMC passes over the shipped step kernels (scripts/pmc_step_kernels.py), each pass its own --pmc run.
# usage: scripts/gpu_pmc_step.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=$1; shift
OUT=$R/gpurun_out/pmcs_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $R/scripts/pmc_step_kernels.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name '*counter_collection.csv' | head -1)
  python3 $R/scripts/pmc_summary.py "$f" --raw > $OUT/p$i.txt
  rm -f "$f"
  cat $OUT/p$i.txt
done
