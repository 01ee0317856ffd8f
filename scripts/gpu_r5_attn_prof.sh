#!/bin/bash
# per-kernel times (kernel trace) of the attention fwd/bwd kernels at the bench shape, then SQ counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/attn_prof${1:+_$1}
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "attention or attn" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/scripts/bench_attn.py --B 4 --S 512 --no-sdpa --iters 20 > $OUT/kt.log 2>&1 || exit 1
python3 $R/scripts/prof_summary.py $(find $OUT/kt -name "*kernel_stats.csv" | head -1) 1 8 | tee $OUT/kt_summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/scripts/bench_attn.py --B 4 --S 512 --no-sdpa --iters 5 > $OUT/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o pmc -- \
  python3 $R/scripts/bench_attn.py --B 4 --S 512 --no-sdpa --iters 5 > $OUT/sq2.log 2>&1 || exit 1
for d in sq sq2; do f=$(find $OUT/$d -name "*counter_collection.csv" | head -1); python3 $R/scripts/pmc_summary.py $f --filter attn --raw; done | tee $OUT/pmc_summary.txt
