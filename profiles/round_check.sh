#!/usr/bin/env bash
# Round-end check on a GPU box (run from the repo root via gpurun):
#   bash profiles/round_check.sh <tag>
# the whole GPU suite, smoke(), the default bench line, then the rocprof
# passes of run_profile.sh; stops at the first failing step.
set -euo pipefail
TAG=${1:-r3d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/${TAG}_gputests.log" 2>&1 \
  || { tail -30 "gpurun_out/${TAG}_gputests.log"; exit 1; }
tail -2 "gpurun_out/${TAG}_gputests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python bench.py > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err"
cat "gpurun_out/${TAG}_bench.json"
timeout -k 10 700 bash profiles/run_profile.sh "$TAG" > "gpurun_out/${TAG}_prof.log" 2>&1
tail -3 "gpurun_out/${TAG}_prof.log"
