#!/usr/bin/env bash
# round-4 call b: RCCL tests, config-5 quality probe, memory-unit counter list
set -uo pipefail
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiprocess.py -k "rccl" > $O/rccl_tests.txt 2>&1 || exit 1
timeout -k 10 500 python -u profiles/probes/quality_probe.py > $O/quality.json 2> $O/quality.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters_list.txt 2>&1 || true
