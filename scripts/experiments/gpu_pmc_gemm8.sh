#!/bin/bash
# PMC passes (own runs, --pmc only) for the gemm8 driver: SQ pass + TCC pass
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_gemm8
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/experiments/gemm8_pmc_driver.py "$@" > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/tcc -o pmc -- \
  python3 $R/scripts/experiments/gemm8_pmc_driver.py "$@" > $OUT/tcc.log 2>&1 || exit 1
for d in sq tcc; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f > $OUT/$d.summary.txt; cat $OUT/$d.summary.txt; done
