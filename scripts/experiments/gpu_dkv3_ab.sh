#!/bin/bash
# dK/dV kernel A/B at D = 128: per-kernel times (kernel trace) of the 32x32x16 form (attn_bwd_dkv128_k) vs the
# 16x16x32 8-wave form (LIPA_ATTN_DKV128=0), each with the split policy auto / forced on
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dkv3_ab${1:+_$1}
mkdir -p $OUT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for shape in "4 512" "2 512" "1 2048"; do
  set -- $shape
  for cfg in ${CFGS:-"1,-1" "1,1" "0,-1" "0,1"}; do   # kernel,split (LIPA_ATTN_DKV128, LIPA_ATTN_DKV_SPLIT)
    IFS=, read v sp <<< "$cfg"
    tag=B$1_S$2_v${v}_s${sp}
    LIPA_ATTN_DKV128=$v LIPA_ATTN_DKV_SPLIT=$sp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o kt -- \
      python3 $R/scripts/bench_attn.py --B $1 --S $2 --no-sdpa --iters 20 > $OUT/$tag.log 2>&1 || exit 1
    echo "== $tag $(tail -1 $OUT/$tag.log)"
    python3 $R/scripts/prof_summary.py $(find $OUT/$tag -name "*kernel_stats.csv" | head -1) 1 6
  done
done 2>&1 | tee $OUT/summary.txt
