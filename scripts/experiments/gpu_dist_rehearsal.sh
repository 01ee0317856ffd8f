#!/bin/bash
# multi-rank rehearsal of the distributed bench on ONE GPU: 2 ranks share cuda:0 (LIPA_SHARE_GPU=1) over
# gloo (RCCL refuses two ranks on one device) — exercises DDP bucket hooks / ZeRO-3 partitioning with the
# real HIP kernels; the RCCL transport itself is the driver's 8-GPU run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0 LIPA_DIST_BACKEND=gloo LIPA_SHARE_GPU=1
mkdir -p $R/gpurun_out/dist
timeout -k 10 400 python3 $R/bench.py --gpus 2 --steps 4 --warmup 2 > $R/gpurun_out/dist/ddp2.log 2>&1; rc=$?
tail -3 $R/gpurun_out/dist/ddp2.log; echo "ddp rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 $R/bench.py --gpus 2 --steps 3 --warmup 1 --strategy zero3 > $R/gpurun_out/dist/z3.log 2>&1; rc=$?
tail -3 $R/gpurun_out/dist/z3.log; echo "zero3 rc=$rc"
exit $rc
