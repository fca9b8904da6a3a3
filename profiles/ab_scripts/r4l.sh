#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forward or dedupe or compaction or plan or user" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
bash _ab/ab_env.sh "NRMS_X=1" "NRMS_SCORE_FOLD=0" "NRMS_SPLIT_CLASSIFY=0" "NRMS_SCORE_FOLD=0 NRMS_SPLIT_CLASSIFY=0" > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
