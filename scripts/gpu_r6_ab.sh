#!/bin/bash
# same-box A/B of the in-tree build against ab_variants/<name> (scripts/ab_variant.sh): alternating default bench runs
# without sub-records.  usage: scripts/gpu_r6_ab.sh <name> [rounds]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0
NAME=$1; N=${2:-3}
O=$R/gpurun_out/ab_$NAME; mkdir -p $O
ARGS="--steps ${STEPS:-20} --warmup 3 --faithful-steps ${FSTEPS:-0} --selective-steps 0 --host-steps 0"
for i in $(seq 1 $N); do
  for v in tree $NAME; do
    if [ $v = tree ]; then B=$R/bench.py; else B=$R/ab_variants/$NAME/bench.py; fi
    timeout -k 10 300 python3 $B $ARGS > $O/$v.$i.json 2> $O/$v.$i.err || { echo "$v run $i failed"; tail -5 $O/$v.$i.err; exit 1; }
    echo "$v $i: $(grep -h '\[bench\]' $O/$v.$i.err | grep -v built | grep -v first | tr '\n' ' ')"
  done
done
