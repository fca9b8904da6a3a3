#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "user or forward" > $O/tests.txt 2>&1 || exit 1
bash _ab/ab_stage.sh _ab/lib_uoold.so _ab/lib_uonew.so > $O/ab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --steps 30 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
