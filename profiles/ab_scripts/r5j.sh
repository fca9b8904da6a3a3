#!/usr/bin/env bash
# r5j: W-resident vocabulary projection (proj_wres_kernel) -- tests, then A/B against the streamed kernel
set -uo pipefail
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "qkv_project or wres or plan_matches or forward or fallback" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash _ab/ab_env.sh "NRMS_PROJ_WRES=0" "NRMS_PROJ_WRES=1" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
