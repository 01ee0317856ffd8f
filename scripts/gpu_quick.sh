#!/bin/bash
# tests touching the LoRA / linear path + 2 bench runs + kernel trace.  usage: scripts/gpu_quick.sh <tag>
export PYTHONPATH=.
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lt_ or lora" tests/test_trainer_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}1.json 2>>gpurun_out/bench_${TAG}.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}2.json 2>>gpurun_out/bench_${TAG}.err &&
bash scripts/gpu_prof.sh $TAG > /dev/null 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${TAG}1.json gpurun_out/bench_${TAG}2.json; exit $rc
