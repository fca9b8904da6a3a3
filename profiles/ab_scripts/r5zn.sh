#!/usr/bin/env bash
# r5zn: UserEncoder wave priority placements, x3 alternated against HEAD:
#   lib_ufprio2 - priority 2 outside the additive GEMM phase, 0 inside (r5zm)
#   lib_ufatt   - priority 2 over staging + attention, 0 from then on
#   lib_uftail  - priority 2 from the softmax on (softmax, pooling, scores)
set -uo pipefail
O=gpurun_out/r5zn; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
for r in 1 2 3; do
  for lib in $L _ab/lib_ufprio2.so _ab/lib_ufatt.so _ab/lib_uftail.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
