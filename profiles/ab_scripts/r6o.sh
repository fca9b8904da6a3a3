#!/usr/bin/env bash
# r6o: news kernel N-tile-12 ownership by bucket (waves holding no N-tile-12 work
# point its W_add fragment loads out of range; NB <= 2 groups give it to wave
# 3; "low": NB <= 2 by the NB >= 3 rule). First try (r6o): branches around
# the loads and MFMAs, 12 % slower. r6o2: branch-free. Parity tests, then an
# A/B against the r6n build (lib_x12old) on one box
set -uo pipefail
O=gpurun_out/r6o${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -5 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['stages_ms']['news_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run new NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run old NRMS_LIB_PATH=$REPO/_ab/lib_x12old.so
  run low NRMS_LIB_PATH=$REPO/_ab/lib_x12low.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
