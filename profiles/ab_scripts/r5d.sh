#!/usr/bin/env bash
# r5d: news kernel C-phase max / NaN rewrite + v_rcp_f32 normalisation (main pass) vs HEAD
set -uo pipefail
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -k "forward or dedupe or compaction or news or overflow or underflow or f16x3 or flow" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -n 1 $O/tests.txt
bash _ab/ab_stage.sh _ab/lib_nfbase.so _ab/lib_cur.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
bash _ab/ab_stage.sh _ab/lib_nfbase.so _ab/lib_cur.so >> $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
