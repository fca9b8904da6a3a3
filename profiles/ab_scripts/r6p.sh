#!/usr/bin/env bash
# r6p: split-f16 projection on three products where no W column fits in 11
# bits (proj_x6.hip): the whole GPU suite, then an A/B on one box of the new
# library (default: three products for the bench's random weights), the same
# library with NRMS_PROJ_PRODUCTS=4, and the r6n build (_ab/lib_x12old.so)
set -uo pipefail
O=gpurun_out/r6p${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -15 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ]; then exit $rc; fi
grep -h "three products" -r $O/gputests.log || true
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['qkv_news'], s['qkv_user'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run new NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run new_p4 NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so NRMS_PROJ_PRODUCTS=4
  run old NRMS_LIB_PATH=$REPO/_ab/lib_x12old.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
