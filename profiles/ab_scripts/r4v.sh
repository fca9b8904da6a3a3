#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4v; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_url.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/tests_url.txt 2>&1 || { tail -30 $O/tests_url.txt; exit 1; }
tail -n 1 $O/tests_url.txt
bash _ab/ab_stage.sh _ab/lib_cur.so _ab/lib_url.so > $O/ab.txt 2>&1 || exit 1
bash _ab/ab_stage.sh _ab/lib_cur.so _ab/lib_url.so >> $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
