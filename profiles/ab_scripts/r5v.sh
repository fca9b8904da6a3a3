#!/usr/bin/env bash
# r5v: the news kernel's two round-5 edits separated, bench stages x3 alternated:
#   HEAD; lib_repfma2 (HEAD + the main pass's rep copies in one fma);
#   lib_rechk (HEAD + recheck pass loading its own group's slices, no scratch); lib_repfma (both)
set -uo pipefail
O=gpurun_out/r5v; mkdir -p $O
L=_ab/lib_head.so
NRMS_LIB_PATH=_ab/lib_repfma2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compaction or news_vectors_golden or fused_news or overflow" > $O/repfma2_tests.log 2>&1 || { tail -30 $O/repfma2_tests.log; exit 1; }
tail -1 $O/repfma2_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_repfma2.so _ab/lib_rechk.so _ab/lib_repfma.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
