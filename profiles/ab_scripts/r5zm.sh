#!/usr/bin/env bash
# r5zm: wave priority (s_setprio) A/B, x3 alternated against HEAD:
#   lib_pxprio  - projection: priority 1 over each k-step's MFMA cluster
#   lib_ufprio  - UserEncoder: priority 2 over the additive GEMM phase
#   lib_ufprio2 - UserEncoder: priority 2 outside the GEMM phase, 0 inside
set -uo pipefail
O=gpurun_out/r5zm; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
for r in 1 2 3; do
  for lib in $L _ab/lib_pxprio.so _ab/lib_ufprio.so _ab/lib_ufprio2.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
