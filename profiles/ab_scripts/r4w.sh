#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "many_classification_blocks or plan_matches" > $O/tests.txt 2>&1; echo "rc=$?"; tail -n 12 $O/tests.txt
