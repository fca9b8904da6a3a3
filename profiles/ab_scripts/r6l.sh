#!/usr/bin/env bash
# r6l: why the r6k build's UserEncoder was slower in every form: HEAD (paired
# path, 4-key groups, 56 KB of code, 128 VGPRs + 28 B scratch) in its default
# and NRMS_USER_PAIR=0 forms, lib_uprolled (paired path, one key per rolled
# iteration, 54 KB, no scratch), lib_upair1 (paired path at occupancy 3),
# lib_unopair4 / lib_unopair1 (no paired code: the r6j kernel, 42.7 KB)
set -uo pipefail
O=gpurun_out/r6l; mkdir -p $O
REPO=$(pwd)
H=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['stages_ms']['user_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run head NRMS_LIB_PATH=$H
  run head_pair0 NRMS_LIB_PATH=$H NRMS_USER_PAIR=0
  run uprolled NRMS_LIB_PATH=$REPO/_ab/lib_uprolled.so
  run upair1 NRMS_LIB_PATH=$REPO/_ab/lib_upair1.so
  run unopair4 NRMS_LIB_PATH=$REPO/_ab/lib_unopair4.so
  run unopair1 NRMS_LIB_PATH=$REPO/_ab/lib_unopair1.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
