#!/bin/bash
# the multi-adapter LoRA kernels in isolation (scripts/bench_lora_multi.py) + two PMC passes over them
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/lora_multi_pmc; mkdir -p $OUT
timeout -k 10 200 python3 $R/scripts/bench_lora_multi.py > $OUT/bench.txt 2>&1 || { tail -5 $OUT/bench.txt; exit 1; }
cat $OUT/bench.txt
[ "${NOPMC:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $R/scripts/bench_lora_multi.py --pmc > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name '*counter_collection.csv' | head -1)
  python3 $R/scripts/pmc_summary.py "$f" --raw > $OUT/p$i.txt
  rm -f "$f"
  cat $OUT/p$i.txt
done
