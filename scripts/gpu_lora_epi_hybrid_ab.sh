#!/bin/bash
# headline step under the hybrid GEMM default: the LoRA terms in the gemm4w q|k|v prologues (LIPA_LORA_EPI=1,
# default) vs hipBLASLt for q|k|v too with the separate LoRA kernels (lora_apply, lora_dx2 as the dX GEMM's C)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/epi_hyb; mkdir -p $O
cd $R
for i in 1 2 3; do
  for e in 1 0; do
    timeout -k 10 300 env LIPA_LORA_EPI=$e python bench.py --faithful-steps 0 --steps 10 --warmup 3 > $O/e$e.$i.json 2> $O/e$e.$i.err || { tail -5 $O/e$e.$i.err; exit 1; }
    echo "lora_epi=$e $i $(grep -o '"ms_per_step": [0-9.]*' $O/e$e.$i.json)"
  done
done
