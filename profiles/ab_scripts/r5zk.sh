#!/usr/bin/env bash
# r5zk: on HEAD (classified-title template + rep fma), with the product's flags,
# x3 alternated:
#   lib_h2rechk - the recheck pass loading its own group's slices (no scratch)
#   lib_h2url   - the UserEncoder row-list chunks on the last workgroups
# after the recheck / overflow and forward tests
set -uo pipefail
O=gpurun_out/r5zk; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_h2rechk.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "overflow or raw_exp or recheck or nan" > $O/h2rechk_tests.log 2>&1 || { tail -30 $O/h2rechk_tests.log; exit 1; }
tail -1 $O/h2rechk_tests.log
NRMS_LIB_PATH=_ab/lib_h2url.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "forward or plan or user or dedupe" > $O/h2url_tests.log 2>&1 || { tail -30 $O/h2url_tests.log; exit 1; }
tail -1 $O/h2url_tests.log
for r in 1 2 3; do
  for lib in $L _ab/lib_h2rechk.so _ab/lib_h2url.so; do
    out=$(NRMS_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2].split('/')[-1], d['value'], d['stages_ms'])" "$out" "$lib" | tee -a $O/ab_stage.txt
  done
done
