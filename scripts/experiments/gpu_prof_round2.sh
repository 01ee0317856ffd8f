#!/bin/bash
# round-2 end-state evidence for the headline step: kernel trace (step timeline) + DRAM traffic per
# kernel (FETCH_SIZE and WRITE_SIZE in their own --pmc passes) + SQ counters (MFMA busy, wait fractions)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_r2
mkdir -p $OUT
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $R/bench.py --steps 3 --warmup 1 > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/sq -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 1 > $OUT/sq.log 2>&1 || exit 1
KT=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/step_timeline.py $KT --marker adamw8bit > $OUT/timeline.txt
python3 $R/scripts/hbm_summary.py $KT $(find $OUT/fetch -name "*counter_collection.csv" | head -1) \
  $(find $OUT/write -name "*counter_collection.csv" | head -1) --top 30 > $OUT/hbm.txt
python3 $R/scripts/pmc_summary.py $(find $OUT/sq -name "*counter_collection.csv" | head -1) > $OUT/sq.txt
cat $OUT/bench.json; head -5 $OUT/timeline.txt; head -12 $OUT/hbm.txt; cp $KT $OUT/trace_keep.csv 2>/dev/null; true
rm -rf $OUT/kt $OUT/fetch $OUT/write $OUT/sq   # raw CSVs exceed gpurun's copy-back cap
