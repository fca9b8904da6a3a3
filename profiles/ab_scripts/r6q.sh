#!/usr/bin/env bash
# r6q: the projection's A planes staged as [2^11 hi | lo | r] with the W lo
# plane packed at 2^-11 (no operand formed in registers) against r6p's
# three-product build (lib_p3mul: 2^11 hi formed per k-step): parity tests,
# then an A/B on one box
set -uo pipefail
O=gpurun_out/r6q${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -5 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['qkv_news'], s['qkv_user'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run new NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run p3mul NRMS_LIB_PATH=$REPO/_ab/lib_p3mul.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
