#!/usr/bin/env bash
# r6t: news kernel groups past a workgroup's first four claimed from a launch
# counter (dynamic balance) against the static stride (lib_nstatic: HEAD's
# news_fused.hip in the same library): parity tests, the balance probe, then
# an A/B on one box
set -uo pipefail
O=gpurun_out/r6t${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -5 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ]; then exit $rc; fi
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -mllvm -amdgpu-sched-strategy=max-ilp profiles/probes/news_variants.hip -o /tmp/nv || exit 1
# (the probe exits 3 here: with NV_ONLY_H3 its f32 reference output is never written)
NV_ONLY_H3=1 timeout -k 10 120 /tmp/nv 56320 5 > $O/nv_balance.txt 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then cat $O/nv_balance.txt; exit $rc; fi
grep -E "kernel avg|workgroup totals" $O/nv_balance.txt
run() {  # tag, env...
  local tag=$1; shift
  out=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['news_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run dyn NRMS_LIB_PATH=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run static NRMS_LIB_PATH=$REPO/_ab/lib_nstatic.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
