#!/usr/bin/env bash
# r5zh: the news kernel templated on classified titles (lib_cls: the per-group
# row staging without run-time branches on the title set; SGPR spills 126 -> 96,
# static v_readlane 733 -> 431) against HEAD: news tests in all arithmetics,
# then bench stages x3 alternated
set -uo pipefail
O=gpurun_out/r5zh; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_cls.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "news or compaction or forward or golden or overflow or dedupe or recheck" > $O/cls_tests.log 2>&1 || { tail -30 $O/cls_tests.log; exit 1; }
tail -1 $O/cls_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_cls.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
