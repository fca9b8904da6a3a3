#!/usr/bin/env bash
# r7c: the news recheck pass folded into the main launch (run by the last
# workgroup to finish, a noinline call) against HEAD's separate recheck
# launch (lib_sep), and (r7c2) the fence on flagging workgroups only against
# no fence at all (lib_nofence, measurement only): the whole GPU suite on the product build (the overflow /
# NaN recheck fixtures), then an A/B on one box
set -uo pipefail
O=gpurun_out/r7c${TAG:-}; mkdir -p $O
REPO=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -2 $O/gputests.log; if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, lib
  local tag=$1; shift
  out=$(NRMS_LIB_PATH=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 100 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], s['news_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run fold $REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run sep $REPO/_ab/lib_sep.so
  run nofence $REPO/_ab/lib_nofence.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
