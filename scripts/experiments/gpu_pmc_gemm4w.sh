#!/bin/bash
# PMC passes (own runs, --pmc only) for the gemm4w driver: two SQ passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-pmc_gemm4w}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/experiments/gemm4w_pmc_driver.py "$@" > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_MFMA_MOPS_BF16 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_DATA_FIFO_FULL --output-format csv -d $OUT/sq2 -o pmc -- \
  python3 $R/scripts/experiments/gemm4w_pmc_driver.py "$@" > $OUT/sq2.log 2>&1 || exit 1
for d in sq sq2; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py --raw $f > $OUT/$d.summary.txt; cat $OUT/$d.summary.txt; done
