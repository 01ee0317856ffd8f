#!/bin/bash
# int4 prefill path (expansion + bf16 GEMM at M >= 1024): quant GPU tests, BASELINE #5 end to end, and the
# headline step native (gemm4w everywhere) vs LIPA_GEMM=lt (hipBLASLt for the bf16 GEMMs), interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/w4_e2e; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for g in native lt; do
    timeout -k 10 300 env LIPA_GEMM=$g python bench.py --faithful-steps 0 --steps 10 --warmup 3 > $O/head_$g$i.json 2> $O/head_$g$i.err || { tail -5 $O/head_$g$i.err; exit 1; }
    echo "head $g $i $(grep -o '"ms_per_step": [0-9.]*' $O/head_$g$i.json)"
  done
done
bash scripts/gpu_awq.sh w4e2e
