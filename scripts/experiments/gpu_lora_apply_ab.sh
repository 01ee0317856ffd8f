#!/bin/bash
# LoRA apply-form A/B: tests, then alternating bench runs, then a kernel trace of the apply step
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora" tests/test_trainer_gpu.py tests/test_quant_gpu.py > gpurun_out/lora_tests.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_apply$i.json 2>>gpurun_out/bench_apply.err &&
  LIPA_LORA_APPLY=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_noapply$i.json 2>>gpurun_out/bench_apply.err || exit 1
done &&
bash scripts/gpu_prof.sh apply > /dev/null 2>&1
rc=$?; tail -2 gpurun_out/lora_tests.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_apply1.json gpurun_out/bench_noapply1.json gpurun_out/bench_apply2.json gpurun_out/bench_noapply2.json; exit $rc
