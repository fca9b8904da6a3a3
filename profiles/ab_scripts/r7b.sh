#!/usr/bin/env bash
# r7b: what the (almost always empty) news recheck launch costs the step: the
# product (16-workgroup grid) against a 1-workgroup grid and no launch at all
# (measurement only: the bench batch flags no title)
set -uo pipefail
O=gpurun_out/r7b; mkdir -p $O
REPO=$(pwd)
run() {  # tag, lib
  local tag=$1; shift
  out=$(NRMS_LIB_PATH=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 100 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], s['news_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run grid16 $REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run grid1 $REPO/_ab/lib_rk1.so
  run none $REPO/_ab/lib_rk0.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
