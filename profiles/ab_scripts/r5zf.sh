#!/usr/bin/env bash
# r5zf: UserEncoder GEMM with its W fragments four k-steps in flight for up to
# two M-tiles (lib_wd4, NRMS_USER_WDEPTH=4; 126 VGPRs, still two workgroups
# per CU) against HEAD: user tests, then bench stages x3 alternated
set -uo pipefail
O=gpurun_out/r5zf; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_wd4.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "user or forward" > $O/wd4_tests.log 2>&1 || { tail -30 $O/wd4_tests.log; exit 1; }
tail -1 $O/wd4_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_wd4.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
