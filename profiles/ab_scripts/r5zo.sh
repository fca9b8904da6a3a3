#!/usr/bin/env bash
# r5zo: wave priority by wave index (waves 0..NW/2-1 one level above their
# SIMD partner), x3 alternated against HEAD (UserEncoder priority 2 / GEMM 0):
#   lib_pxpar - projection: waves 0-3 priority 1
#   lib_ufpar - UserEncoder: waves 0-3 one level above waves 4-7 (3/1 vs 2/0)
set -uo pipefail
O=gpurun_out/r5zo; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
for r in 1 2 3; do
  for lib in $L _ab/lib_pxpar.so _ab/lib_ufpar.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
