#!/bin/bash
# round-5 check: GPU tests of the touched paths (or all with K=), smoke(), the default bench, a kernel trace of
# the headline step.  usage: scripts/gpu_r5_check.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-a}
O=$R/gpurun_out/r5check_$TAG; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_trainer_gpu.py tests/test_optin_paths_gpu.py tests/test_lora_multi_gpu.py tests/test_dist_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; tail -1 $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -1 $O/bench.json; grep "\[bench\]" $O/bench.err; [ $rc -eq 0 ] || exit $rc
[ "${PROF:-1}" = 1 ] && bash scripts/gpu_step_prof.sh r5$TAG
exit 0
