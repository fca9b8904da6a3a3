#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fallback_without_tail or many_classification" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.txt
