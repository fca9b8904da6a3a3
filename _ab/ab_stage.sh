#!/usr/bin/env bash
# One bench.py run (no extras) per library, alternated x2: prints the per-stage ms.
#   bash _ab/ab_stage.sh <libA.so> <libB.so> ...
set -euo pipefail
for rep in 1 2; do
  for lib in "$@"; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib"
  done
done
