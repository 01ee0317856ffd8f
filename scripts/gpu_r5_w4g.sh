#!/bin/bash
# w4g (int4 W4A16 for decode batches 33..64): numerics, microbench vs bf16 / w4mm / gemm4w W4=2, then BASELINE #5
# end to end (merged-LoRA Qwen3-8B, bf16 vs int4 RTN g128: decode per batch + 4 x 512 prefill)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
OUT=$R/gpurun_out/w4g${1:+_$1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $R/tests/test_quant_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u $R/scripts/bench_w4.py 32 48 64 128 256 > $OUT/bench_w4.txt 2>&1 || { tail -20 $OUT/bench_w4.txt; exit 1; }
python3 - $OUT/bench_w4.txt <<'PY' | tee $OUT/bench_w4_summary.txt
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    r = json.loads(l)
    ks = " ".join(f'{k[4:]}={v}' for k, v in r.items() if k.startswith("w4g_ks") and k != "w4g_ks")
    print(f'{r["shape"]:8s} M={r["M"]:4d} bf16 {r["bf16_us"]:7.1f} g4w {r.get("bf16_g4w_us", 0):7.1f} | w4g {r.get("w4g_us", 0):7.1f} (ks {r.get("w4g_ks")}, err {r.get("w4g_relerr", 0):.4f}; {ks}) w4mm {r.get("w4mm_us", 0):7.1f} g4w_int4 {r.get("g4w_int4_us", 0):7.1f} expand+g4w {r.get("expand_g4w_us", 0):7.1f}')
PY
timeout -k 10 600 python -u -m llm_in_practise_amd.bench.awq_infer --method rtn --batches 1 8 32 48 64 128 256 \
  --ppl-prompts 1 --ppl-new 8 --out $OUT/awq.json > $OUT/awq.log 2>&1 || { tail -30 $OUT/awq.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/awq.json')); print('speedup', d['decode_speedup']); print('prefill bf16', d['bf16']['prefill']['ms'], 'int4', d['int4']['prefill']['ms'])"
