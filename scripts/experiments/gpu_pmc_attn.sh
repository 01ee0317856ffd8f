#!/bin/bash
# attention kernels at the bench shape: PMC passes (own runs, --pmc only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_attn
mkdir -p $OUT
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "qk_norm or attn or lora" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/bench_attn.py --B 4 --S 512 > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o pmc -- \
  python3 $R/scripts/bench_attn.py --B 4 --S 512 > $OUT/sq2.log 2>&1 || exit 1
for d in sq sq2; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f --filter attn --raw > $OUT/$d.summary.txt; cat $OUT/$d.summary.txt; done
