#!/usr/bin/env bash
# r6x: the three-product projection on two-plane A tiles of 80 / 96 / 112 rows
# (product: 96) against HEAD's 64-row three-plane tiles (lib_g64): the
# projection parity tests on the product build, then an A/B on one box
set -uo pipefail
O=gpurun_out/r6x${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -2 $O/gputests.log; if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['qkv_news'], s['qkv_user'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run g96 NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run g64 NRMS_LIB_PATH=$REPO/_ab/lib_g64.so
  run g80 NRMS_LIB_PATH=$REPO/_ab/lib_g80.so
  run g112 NRMS_LIB_PATH=$REPO/_ab/lib_g112.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
