#!/usr/bin/env bash
# r6w: projection tile height probe: 32-row A tiles (twice the items, half
# the rows per W fragment read) against the 64-row product build, to see how
# much of qkv_news / qkv_user is per-item overhead
set -uo pipefail
O=gpurun_out/r6w; mkdir -p $O
REPO=$(pwd)
NRMS_LIB_PATH=$REPO/_ab/lib_pm32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "qkv_project" --timeout 200 --timeout-method thread > $O/pm32_tests.log 2>&1
rc=$?; tail -2 $O/pm32_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['qkv_news'], s['qkv_user'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run pm64 NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run pm32 NRMS_LIB_PATH=$REPO/_ab/lib_pm32.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
