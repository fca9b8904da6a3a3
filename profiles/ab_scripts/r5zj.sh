#!/usr/bin/env bash
# r5zj: news-kernel variants rebuilt with the product's per-file flags (max-ILP
# scheduler; earlier variant builds of news_fused.hip had the default
# scheduler), x3 alternated against HEAD:
#   lib_hfma - the main pass's rep copies in one fma
#   lib_hdef - HEAD under the default machine scheduler
#   lib_htup - the title-set pointers out of their SGPR tuple, recheck list from the counters
set -uo pipefail
O=gpurun_out/r5zj; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_hfma.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compaction or news_vectors_golden or fused_news or overflow" > $O/hfma_tests.log 2>&1 || { tail -30 $O/hfma_tests.log; exit 1; }
tail -1 $O/hfma_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_hfma.so _ab/lib_hdef.so _ab/lib_htup.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
