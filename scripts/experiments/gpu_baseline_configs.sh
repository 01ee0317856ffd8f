#!/bin/bash
# BASELINE.json configs #2, #3 (reference-faithful) and #5 on one MI355X; results under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
# 2: Qwen3-8B LoRA bf16 (Fine-Tuning/qwen3-8b-lora.py:128-170: r16/a32/drop .05 on q,k,v,o; bs2 x GA4; adamw_torch; ckpt)
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --mode lora --targets q_proj,k_proj,v_proj,o_proj \
  --lora-r 16 --lora-alpha 32 --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 --grad-ckpt \
  > gpurun_out/cfg2_lora_ckpt.json 2> gpurun_out/cfg2.err &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --mode lora --targets q_proj,k_proj,v_proj,o_proj \
  --lora-r 16 --lora-alpha 32 --lora-dropout 0.05 --grad-accum 4 --optim adamw_torch --lr 1e-4 \
  > gpurun_out/cfg2_lora_tuned.json 2>> gpurun_out/cfg2.err &&
# 3: QLoRA headline, reference-faithful (gradient checkpointing on, sequential GA) beside the tuned default
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --grad-ckpt --ga-fusion 0 \
  > gpurun_out/cfg3_qlora_faithful.json 2> gpurun_out/cfg3.err &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/cfg3_qlora_tuned.json 2>> gpurun_out/cfg3.err &&
# 5: merged adapter -> AWQ int4 W4A16 inference (decode / prefill / serving / quality vs bf16)
timeout -k 10 700 python -m llm_in_practise_amd.bench.awq_infer --model qwen3-8b --method awq \
  --serve-requests 256 --out gpurun_out/cfg5_awq.json > gpurun_out/cfg5.log 2>&1
rc=$?
cat gpurun_out/cfg2_lora_ckpt.json gpurun_out/cfg2_lora_tuned.json gpurun_out/cfg3_qlora_faithful.json \
  gpurun_out/cfg3_qlora_tuned.json 2>/dev/null
tail -c 1500 gpurun_out/cfg5.log
exit $rc
