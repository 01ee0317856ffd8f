#!/bin/bash
# PyTorch TunableOp over hipBLASLt/rocBLAS for the bench's GEMM shapes: tune (resuming from the
# committed configs/tunableop CSV), then A/B the bench with and without the tuned selections.
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=$PWD/gpurun_out/tunableop
mkdir -p $D
cp configs/tunableop/tunableop_results0.csv $D/ 2>/dev/null || true
export PYTORCH_TUNABLEOP_FILENAME=$D/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=25 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30
export PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 PYTORCH_TUNABLEOP_MAX_WARMUP_ITERATIONS=3
( while sleep 45; do echo "[tune] $(date +%T) $(wc -l < $D/tunableop_results0.csv 2>/dev/null) lines"; done ) &
PROG=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python bench.py --steps 2 --warmup 2 \
  > $D/tune.log 2>&1; rc=$?
kill $PROG
[ $rc -eq 0 ] || { tail -20 $D/tune.log; exit 1; }
grep "ms/step" $D/tune.log
wc -l $D/*.csv
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $D/off.log 2>&1 || exit 1
  echo "default  $(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' $D/off.log)"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --steps 8 --warmup 2 \
    > $D/on.log 2>&1 || { tail -20 $D/on.log; exit 1; }
  echo "tuned    $(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' $D/on.log)"
done
