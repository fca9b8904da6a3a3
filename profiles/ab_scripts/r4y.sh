#!/usr/bin/env bash
set -euo pipefail
TAG=r4y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/${TAG}_gputests.log" 2>&1 || { tail -30 "gpurun_out/${TAG}_gputests.log"; exit 1; }
tail -2 "gpurun_out/${TAG}_gputests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python bench.py > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err"
cat "gpurun_out/${TAG}_bench.json" | head -c 600
