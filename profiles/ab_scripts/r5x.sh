#!/usr/bin/env bash
# r5x = r5w (chunked UserEncoder instance) then the news-kernel edits separated:
# HEAD vs lib_repfma2 (rep copies in one fma) vs lib_rechk (recheck pass without scratch), x2
set -uo pipefail
bash profiles/ab_scripts/r5w.sh || exit 1
O=gpurun_out/r5x; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_repfma2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compaction or news_vectors_golden or fused_news or overflow" > $O/repfma2_tests.log 2>&1 || { tail -30 $O/repfma2_tests.log; exit 1; }
tail -1 $O/repfma2_tests.log
for r in 1 2; do
  for lib in _ab/lib_head.so _ab/lib_repfma2.so _ab/lib_rechk.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
