#!/usr/bin/env bash
# r7k: machine-scheduler strategy per file, re-checked after round 6's code
# changes: news_fused.hip under the default scheduler (product: max-ILP),
# proj_x6.hip and user_fused.hip under max-ILP (product: default)
set -uo pipefail
O=gpurun_out/r7k; mkdir -p $O
REPO=$(pwd)
run() {  # tag, lib
  local tag=$1; shift
  out=$(NRMS_LIB_PATH=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 50 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], s['qkv_news'], s['news_fused'], s['qkv_user'], s['user_fused'], d['forward_paths_bitwise_equal'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run product $REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run nf_default $REPO/_ab/lib_nf_default.so
  run px_maxilp $REPO/_ab/lib_px_maxilp.so
  run uf_maxilp $REPO/_ab/lib_uf_maxilp.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
