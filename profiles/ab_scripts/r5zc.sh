#!/usr/bin/env bash
# r5zc: against HEAD, bench stages x3 alternated of
#   lib_urlast - the news kernel's user-row-list chunks on the last workgroups (which have a group fewer)
#   lib_clslds - the title classification's compacted row ids through an LDS row per thread (NRMS_CLS_LDS)
# after their tests
set -uo pipefail
O=gpurun_out/r5zc; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
t() { NRMS_LIB_PATH=_ab/lib_$1.so timeout -k 10 400 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread -k "$3" > $O/$1_tests.log 2>&1 || { tail -30 $O/$1_tests.log; exit 1; }; echo "$1: $(tail -1 $O/$1_tests.log)"; }
t urlast "tests/test_gpu_parity.py tests/test_gpu_flow.py" "forward or plan or user or dedupe"
t clslds "tests/test_gpu_parity.py tests/test_gpu_flow.py" "forward or plan or compaction or dedupe or classif or golden"
for r in 1 2 3; do
  for lib in $L _ab/lib_urlast.so _ab/lib_clslds.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
