#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4t; mkdir -p $O
for e in "NRMS_X=1" "NRMS_SPLIT_CLASSIFY=0" "NRMS_SCORE_FOLD=0" "NRMS_USER_LPT=0"; do
  echo "== $e"
  env NRMS_LIB_PATH=_ab/lib_url.so $e timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "test_forward_golden" > "$O/t_${e%%=*}.txt" 2>&1; echo "rc=$?"
  tail -n 3 "$O/t_${e%%=*}.txt"
done
