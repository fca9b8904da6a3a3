#!/usr/bin/env bash
# r7g: end-of-round-6 build check (launcher relay, determinism test): the whole GPU
# suite, smoke, the driver's default bench line, then the profile recipe
set -uo pipefail
O=gpurun_out/r7g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -15 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['stages_ms'],d['cpu_baseline']['value'],d['roofline']['frac'])"
timeout -k 10 900 bash profiles/run_profile.sh r7g > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -2 $O/profile.log
