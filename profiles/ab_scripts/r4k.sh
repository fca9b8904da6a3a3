#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forward or dedupe or compaction or plan" > $O/tests_cur.txt 2>&1 || { tail -30 $O/tests_cur.txt; exit 1; }
for v in tstart clsfirst tscf; do
  NRMS_LIB_PATH=_ab/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forward or dedupe or compaction or plan" > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
done
tail -1 $O/tests_*.txt
bash _ab/ab_stage.sh _ab/lib_cur.so _ab/lib_tstart.so _ab/lib_clsfirst.so _ab/lib_tscf.so > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
