#!/usr/bin/env bash
# r6k: UserEncoder long users (35..50 titles) with two queries per thread in
# one pass (HEAD default) against two passes split by head (NRMS_USER_PAIR=0)
# and by task index (+ NRMS_USER_HSPLIT=0): the user GPU tests (the three
# forms bitwise equal), same-library env A/B x3, FETCH of fused_user_kernel
set -uo pipefail
O=gpurun_out/r6k; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "user" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 900 bash _ab/ab_env.sh "" "NRMS_USER_PAIR=0" "NRMS_USER_PAIR=0 NRMS_USER_HSPLIT=0" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/$O/pair_F -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/pair_F.log 2>&1 || { echo "pmc failed"; tail -5 $O/pair_F.log; exit 1; }
python profiles/pmc_sum.py $O/pair_F fused_user
