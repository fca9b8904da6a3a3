#!/usr/bin/env bash
# A/B of builds that need their own source tree (e.g. an older ABI): each
# argument is <dir>:<lib> (lib relative to the repo root, or "-" for the
# dir's own in-tree build); bench.py of <dir> runs with that library,
# alternated x2.   bash _ab/ab_dirs.sh _ab/head:- .:-
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for rep in 1 2; do
  for arg in "$@"; do
    d=${arg%%:*}; l=${arg#*:}
    if [ "$l" = "-" ]; then lib=$ROOT/$d/newsrecommendationsystem_amd/libnrms_hip.so; else lib=$ROOT/$l; fi
    out=$(cd "$ROOT/$d" && NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['stages_ms'])" "$out" "$arg"
  done
done
