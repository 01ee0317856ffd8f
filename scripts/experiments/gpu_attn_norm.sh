set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "attention or rmsnorm or qwen3" --timeout 120 --timeout-method thread > gpurun_out/t18.log 2>&1 || { tail -30 gpurun_out/t18.log; exit 1; }
tail -1 gpurun_out/t18.log
timeout -k 10 120 python scripts/bench_attn.py > gpurun_out/attn_bench2.log 2>&1 && cat gpurun_out/attn_bench2.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/q_bench.log 2>&1 || { tail -20 gpurun_out/q_bench.log; exit 1; }
echo "$(grep -o '[0-9.]* ms/step  [0-9,]* tok/s' gpurun_out/q_bench.log)"
done
