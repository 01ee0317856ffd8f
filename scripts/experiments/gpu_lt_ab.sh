#!/bin/bash
# direct hipBLASLt base GEMMs (LIPA_LT=1, default) vs torch.addmm/mm/bmm (LIPA_LT=0): tests,
# alternating bench runs on one box, kernel trace of the new default
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lt_ or lora" tests/test_trainer_gpu.py > gpurun_out/lt_tests.log 2>&1 &&
LIPA_LT_VERBOSE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_lt0.json 2> gpurun_out/bench_lt_verbose.err &&
for i in 1 2; do
  LIPA_LT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_nolt$i.json 2>>gpurun_out/bench_lt.err &&
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_lt$i.json 2>>gpurun_out/bench_lt.err || exit 1
done &&
bash scripts/gpu_prof.sh lt > /dev/null 2>&1
rc=$?; tail -2 gpurun_out/lt_tests.log; grep "\[lt\]" gpurun_out/bench_lt_verbose.err | sort | uniq | head -20
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_lt0.json gpurun_out/bench_nolt1.json gpurun_out/bench_lt1.json gpurun_out/bench_nolt2.json gpurun_out/bench_lt2.json; exit $rc
