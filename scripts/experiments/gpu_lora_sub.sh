set -u; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for S in 1 2; do echo "sub=$S"; LIPA_LORA_SUB=$S timeout -k 10 100 python scripts/bench_lora.py > gpurun_out/lora_s$S.log 2>&1 || exit 1; grep acc_ gpurun_out/lora_s$S.log; done
