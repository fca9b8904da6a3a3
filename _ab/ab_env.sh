#!/usr/bin/env bash
# One bench.py run (no extras) per environment setting, alternated x3: prints the per-stage ms.
#   bash _ab/ab_env.sh "" "NRMS_X=0" "NRMS_Y=0 NRMS_X=0" ...
set -euo pipefail
for rep in 1 2 3; do
  for e in "$@"; do
    out=$(env $e timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(repr(sys.argv[2]), d['value'], d['ms_per_step'], d['stages_ms'])" "$out" "$e"
  done
done
