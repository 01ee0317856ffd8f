#!/bin/bash
# W4A16 at prefill row counts: gemm4w W4=2 (in-kernel table) vs one bf16 expansion (int4_dequant_k) + bf16 gemm4w
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONPATH=$R HSA_ENABLE_IPC_MODE_LEGACY=0
O=$R/gpurun_out/w4_prefill; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/bench_w4.py 128 256 512 1024 2048 4096 > $O/bench.jsonl 2>&1 || { tail -5 $O/bench.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/w4_prefill/bench.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(f"{r['shape']:8s} M={r['M']:5d} bf16 {min(r['bf16_us'], r.get('bf16_g4w_us', 1e9)):8.1f}  W4=2 {r.get('g4w_int4_us', 0):8.1f}  expand {r.get('expand_us', 0):6.1f} + g4w = {r.get('expand_g4w_us', 0):8.1f}  err {r.get('expand_relerr', 0):.1e}")
PY
