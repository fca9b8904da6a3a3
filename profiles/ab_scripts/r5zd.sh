#!/usr/bin/env bash
# r5zd: the projection loading each item's first two k-steps' W fragments in
# the previous item, the second before that item's output stores (lib_b1,
# NRMS_PX_B1AHEAD=1) against HEAD: projection / forward tests in all
# arithmetics, then bench stages x3 alternated
set -uo pipefail
O=gpurun_out/r5zd; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_b1.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "qkv or proj or forward or user" > $O/b1_tests.log 2>&1 || { tail -30 $O/b1_tests.log; exit 1; }
tail -1 $O/b1_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_b1.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
