#!/usr/bin/env bash
# r7l: the UserEncoder under the max-ILP scheduler (build.py FILE_FLAGS): the
# whole GPU suite, the bench logits bitwise against the previous library,
# and an A/B on one box
set -uo pipefail
O=gpurun_out/r7l; mkdir -p $O
REPO=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -2 $O/gputests.log; if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # tag, lib
  local tag=$1; shift
  out=$(NRMS_LIB_PATH=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 50 --dump-logits $O/lg_$tag 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], d['ms_per_step'], s['user_fused'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run maxilp $REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run prev $REPO/_ab/lib_prev.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r7l/lg_maxilp.rank0.npz")["logits"]; b = np.load("gpurun_out/r7l/lg_prev.rank0.npz")["logits"]
print("logits bitwise equal to the previous library:", np.array_equal(a.view(np.uint32), b.view(np.uint32)))
PY
