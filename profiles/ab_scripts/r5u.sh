#!/usr/bin/env bash
# r5u: against HEAD's library, bench stages alternated x2 of
#   lib_rechk   - news recheck pass without scratch (its group's slices loaded at the group start)
#   lib_repfma  - lib_rechk + the main pass's rep copies in one fma (NRMS_REP_FMA)
# after their GPU tests; then the UserEncoder at two workgroups per CU (<32, 512>) vs one
# (<50, 832>, NRMS_USER_LMAX=50) on a 32-title history probe
set -uo pipefail
O=gpurun_out/r5u; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
t() { NRMS_LIB_PATH=_ab/lib_$1.so timeout -k 10 400 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread -k "$3" > $O/$1_tests.log 2>&1 || { tail -30 $O/$1_tests.log; exit 1; }; echo "$1: $(tail -1 $O/$1_tests.log)"; }
t rechk "tests/test_gpu_parity.py tests/test_gpu_flow.py" "overflow or raw_exp or recheck or nan"
t repfma tests/test_gpu_parity.py "compaction or news_vectors_golden or fused_news"
timeout -k 10 400 bash _ab/ab_stage.sh $L _ab/lib_rechk.so _ab/lib_repfma.so > $O/ab_stage.txt 2>&1 || { cat $O/ab_stage.txt; exit 1; }
cat $O/ab_stage.txt
for rep in 1 2; do
  for e in "NRMS_USER_LMAX=0" "NRMS_USER_LMAX=50"; do
    out=$(env $e NRMS_PROBE_CLICKED=32 timeout -k 10 120 python profiles/probes/bench_clicked.py --no-cpu-baseline --no-extras --steps 30 2>/dev/null) || exit 1
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['stages_ms'])" "$out" "$e" | tee -a $O/user_2wg.txt
  done
done
