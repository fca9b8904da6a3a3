#!/usr/bin/env bash
# r6z: projection wave roles. Phase stamps (gpurun_out/r6z/px_waves.txt): the
# 2-tile waves 4-7 (younger, losing issue arbitration) spend 167 k cycles in
# k-steps 1-9 against 133 k for the 3-tile waves 0-3 and arrive last at the
# restage barrier. Variants: swap (waves 0-3 two tiles, 4-7 three), prio47
# (waves 4-7 at s_setprio 1), swapprio (both); the same bench logits are
# checked bitwise against the product library's
set -uo pipefail
O=gpurun_out/r6z; mkdir -p $O
REPO=$(pwd)
run() {  # tag, lib
  local tag=$1; shift
  out=$(NRMS_LIB_PATH=$1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 --dump-logits $O/lg_$tag 2>/dev/null) || { echo "$tag failed"; return 1; }
  python -c "import json,sys; d=json.loads(sys.argv[1]); s=d['stages_ms']; print(sys.argv[2], d['value'], s['qkv_news'], s['qkv_user'])" "$out" "$tag"
}
for rep in 1 2 3; do
  run base $REPO/newsrecommendationsystem_amd/libnrms_hip.so
  run swap $REPO/_ab/lib_swap.so
  run prio47 $REPO/_ab/lib_prio47.so
  run swapprio $REPO/_ab/lib_swapprio.so
done > $O/ab.txt 2>&1
cat $O/ab.txt
python - <<'PY'
import numpy as np
b = np.load("gpurun_out/r6z/lg_base.rank0.npz")["logits"]
for t in ("swap", "prio47", "swapprio"):
    x = np.load(f"gpurun_out/r6z/lg_{t}.rank0.npz")["logits"]
    print(t, "logits bitwise equal to base:", np.array_equal(x.view(np.uint32), b.view(np.uint32)))
PY
