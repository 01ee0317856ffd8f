set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for rep in 1 2 3; do
for b in bench_ab_old.py bench.py; do
timeout -k 10 300 python $b --steps 30 --warmup 5 > gpurun_out/ab_$b.log 2>&1 || exit 1
echo "$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$b.log)"
done
done
bash scripts/gpu_prof.sh v13
