#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4r2; mkdir -p $O
for v in nfilp nfmem; do
  NRMS_LIB_PATH=_ab/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "forward or dedupe or compaction or news" > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -n 1 $O/tests_$v.txt
done
bash _ab/ab_stage.sh _ab/lib_cur.so _ab/lib_nfilp.so _ab/lib_nfmem.so > $O/ab.txt 2>&1 || exit 1
bash _ab/ab_stage.sh _ab/lib_cur.so _ab/lib_nfilp.so _ab/lib_nfmem.so >> $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
