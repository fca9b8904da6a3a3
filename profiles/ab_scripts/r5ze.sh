#!/usr/bin/env bash
# r5ze: as r5zd, the next item's k-step-1 W fragments loaded tile by tile inside
# the interleaved last k-step, each tile's ahead of its stores (lib_b2), against HEAD:
# projection / forward tests, then bench stages x3 alternated
set -uo pipefail
O=gpurun_out/r5ze; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_b2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "qkv or proj or forward or user" > $O/b2_tests.log 2>&1 || { tail -30 $O/b2_tests.log; exit 1; }
tail -1 $O/b2_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_b2.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
