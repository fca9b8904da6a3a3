#!/usr/bin/env bash
# A/B of two bench.py versions on one box (same library): bash _ab/ab_benchpy.sh <a.py> <b.py>
set -euo pipefail
for rep in 1 2 3; do
  for b in "$@"; do
    out=$(timeout -k 10 120 python "$b" --no-cpu-baseline --no-extras --steps 50 2>/dev/null)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['ms_per_step'], round(sum(d['stages_ms'].values()), 4))" "$out" "$b"
  done
done
