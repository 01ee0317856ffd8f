set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for mt in 8 16; do
LIPA_GEMM_MT=$mt timeout -k 10 200 python scripts/bench_gemm.py --m 2048 --iters 20 --quick --impls 3 > gpurun_out/mt$mt.log 2>&1 || exit 1
echo MT=$mt; grep -E "nf4" gpurun_out/mt$mt.log
done
