set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serving_gpu.py tests/test_decode_gpu.py > gpurun_out/serve_tests.log 2>&1 || { tail -30 gpurun_out/serve_tests.log; exit 1; }
tail -3 gpurun_out/serve_tests.log
bash scripts/experiments/gpu_serve_ref.sh
