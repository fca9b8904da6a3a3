#!/usr/bin/env bash
# r6a: round-6 first check: the GPU suite with the tightened tolerances (no -x:
# every failure listed), the self-launching --gpus 2 bench, then the driver's bench command
set -uo pipefail
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
rc=$?
tail -30 $O/gputests.log | grep -E "passed|failed|FAILED|ERROR" || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['stages_ms'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -q -s -k zipf_long --timeout 120 > $O/zipf.log 2>&1 || { tail -20 $O/zipf.log; exit 1; }
grep "embedding backward" $O/zipf.log
