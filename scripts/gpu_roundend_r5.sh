#!/bin/bash
# round-end rehearsal: the whole GPU test tier, smoke(), then the default bench.py (as the driver runs them), each
# step timed.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/roundend_$1; mkdir -p $OUT
cd $R
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations 15 > $OUT/tests.txt 2>&1
rc=$?; tail -22 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
t1=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1
rc=$?; tail -2 $OUT/smoke.txt; [ $rc -eq 0 ] || exit $rc
t2=$(date +%s)
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -1 $OUT/bench.json; grep "\[bench\]" $OUT/bench.err
t3=$(date +%s)
echo "seconds: tests $((t1-t0)) smoke $((t2-t1)) bench $((t3-t2))" | tee $OUT/times.txt
exit $rc
