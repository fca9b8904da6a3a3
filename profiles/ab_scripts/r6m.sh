#!/usr/bin/env bash
# r6m: UserEncoder paired queries (one key per rolled iteration) for users of
# >= 35 titles (HEAD) and, as probes, >= 33 / 25 / 17 titles; lib_unopair4 =
# no paired path (the r6j kernel). User GPU tests on HEAD, then A/B x3.
set -uo pipefail
O=gpurun_out/r6m; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "user" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 1000 bash _ab/ab_bench.sh newsrecommendationsystem_amd/libnrms_hip.so _ab/lib_upmin33.so _ab/lib_upmin25.so _ab/lib_upmin17.so _ab/lib_unopair4.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
