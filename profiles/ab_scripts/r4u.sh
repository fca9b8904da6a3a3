#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4u; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_url.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "user or forward" > $O/t1.txt 2>&1; echo "rc=$?"; tail -n 3 $O/t1.txt
NRMS_LIB_PATH=_ab/lib_url.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "test_user_encode_strided_views_through_c_abi or test_forward_golden" > $O/t2.txt 2>&1; echo "rc=$?"; tail -n 3 $O/t2.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "user or forward" > $O/t3.txt 2>&1; echo "rc=$?"; tail -n 3 $O/t3.txt
