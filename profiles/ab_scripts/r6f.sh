#!/usr/bin/env bash
# r6f: round-6 build check: the whole GPU suite, smoke, the driver's default
# bench line (all extras: gather, config 2, GEMM legs, FedAvg quality, CPU
# baseline, AUC, eval throughput)
set -uo pipefail
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -15 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['stages_ms'],d['cpu_baseline']['value'],d['roofline']['frac'])"
