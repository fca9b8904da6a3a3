#!/usr/bin/env bash
# round-4 first GPU call: bench, user-LPT A/B, RCCL world-1 tests, config-5 quality probe
set -euo pipefail
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
for rep in 1 2 3; do
  for lpt in 1 0; do
    out=$(NRMS_USER_LPT=$lpt timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null)
    python -c "import json,sys; d=json.loads(sys.argv[1]); print('lpt', sys.argv[2], d['value'], d['stages_ms'])" "$out" "$lpt" >> $O/lpt_ab.txt
  done
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "user" > $O/user_tests.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiprocess.py -k "rccl" > $O/rccl_tests.txt 2>&1
timeout -k 10 400 python -u profiles/probes/quality_probe.py > $O/quality.json 2> $O/quality.err
