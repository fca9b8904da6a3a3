#!/usr/bin/env bash
# r5zg: the projection loading its epilogue's bias and column exponents in the
# last k-step pair instead of at the item start (lib_lb, NRMS_PX_LATE_BIAS=1: no
# spills, no scratch) against HEAD: projection / forward tests, then bench stages x3
set -uo pipefail
O=gpurun_out/r5zg; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_lb.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "qkv or proj or forward or user" > $O/lb_tests.log 2>&1 || { tail -30 $O/lb_tests.log; exit 1; }
tail -1 $O/lb_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_lb.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
