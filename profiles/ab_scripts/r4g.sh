#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4g; mkdir -p $O
bash _ab/ab_stage.sh _ab/lib_pxold.so _ab/lib_pxnew.so > $O/proj_ab.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "qkv or forward" > $O/proj_tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u profiles/probes/quality_probe.py > $O/quality.json 2> $O/quality.err || exit 1
