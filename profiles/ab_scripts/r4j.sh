#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
bash _ab/ab_stage.sh _ab/lib_head.so newsrecommendationsystem_amd/libnrms_hip.so _ab/lib_pxeb1.so > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --steps 30 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
