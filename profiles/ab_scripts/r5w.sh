#!/usr/bin/env bash
# r5w: the UserEncoder's 512-thread, 80-KB instance for 33-50-title histories
# (two workgroups per CU; lib_uchunk): its user tests in all arithmetics, then
# bench stages with NRMS_USER_CHUNK=1 / 0 (the 832-thread instance) on the same
# library, x3 alternated
set -uo pipefail
O=gpurun_out/r5w; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_uchunk.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "user or forward or prediction or plan or flow" > $O/uchunk_tests.log 2>&1 || { tail -40 $O/uchunk_tests.log; exit 1; }
tail -1 $O/uchunk_tests.log
for r in 1 2 3; do
  for e in NRMS_USER_CHUNK=1 NRMS_USER_CHUNK=0; do
    out=$(env $e NRMS_LIB_PATH=_ab/lib_uchunk.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['stages_ms'])" "$out" "$e" | tee -a $O/ab_stage.txt
  done
done
