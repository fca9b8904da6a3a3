#!/usr/bin/env bash
# r5zi: the news kernel with its title-set pointers copied out of their 8-SGPR
# argument tuple (one s_mov_b64 each, so a spill reloads one pointer, not the
# tuple) and the recheck list addressed from the counters (lib_tup; v_readlane
# per NB = 5 group 55 -> 32) against HEAD: news tests, then bench stages x3
set -uo pipefail
O=gpurun_out/r5zi; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_tup.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "news or compaction or forward or golden or overflow or dedupe or recheck" > $O/tup_tests.log 2>&1 || { tail -30 $O/tup_tests.log; exit 1; }
tail -1 $O/tup_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_tup.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
