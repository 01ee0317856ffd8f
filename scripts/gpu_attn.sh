#!/bin/bash
# attention: GPU tests, microbench at the bench shape and S=2048, LDS-conflict PMC pass.  usage: scripts/gpu_attn.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=$1
OUT=$R/gpurun_out/attn_$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "attention or attn" > $OUT/tests.txt 2>&1
rc=$?; tail -3 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u $R/scripts/bench_attn.py > $OUT/bench.txt 2>&1 && \
timeout -k 10 200 python -u $R/scripts/bench_attn.py --B 1 --S 2048 >> $OUT/bench.txt 2>&1
rc=$?; cat $OUT/bench.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p -o pmc -- python3 $R/scripts/bench_attn.py > $OUT/p.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p.log; exit 1; }
f=$(find $OUT/p -name '*counter_collection.csv' | head -1)
python3 $R/scripts/pmc_summary.py "$f" --filter attn --raw > $OUT/pmc.txt; rm -f "$f"; cat $OUT/pmc.txt
