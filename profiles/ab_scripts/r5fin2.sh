#!/usr/bin/env bash
# r5fin2: round-5 final build check (+ UserEncoder wave priority), then the r5zo A/B: full GPU suite, smoke, the driver's bench
# command,
set -uo pipefail
O=gpurun_out/r5fin2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['stages_ms'])"
bash profiles/ab_scripts/r5zo.sh
