#!/usr/bin/env bash
# r6j: UserEncoder head split, each pass staging only its own heads: first
# pass of up to 10 heads (HEAD), of 8 only (lib_userhs8), 8 or 10
# (lib_userhs810), against the round-5 task-index split; the user GPU tests,
# bench A/B x3, FETCH of fused_user_kernel per library
set -uo pipefail
O=gpurun_out/r6j; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "user" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
H=newsrecommendationsystem_amd/libnrms_hip.so
timeout -k 10 1000 bash _ab/ab_bench.sh $H _ab/lib_userhs8.so _ab/lib_userhs810.so _ab/lib_user_r5.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for lib in $H _ab/lib_userhs8.so _ab/lib_userhs810.so; do
  tag=$(basename $lib .so)
  ( cd /tmp && export TMPDIR=/tmp && NRMS_LIB_PATH=$REPO/$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/$O/${tag}_F -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/${tag}_F.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/${tag}_F.log; exit 1; }
  python profiles/pmc_sum.py $O/${tag}_F fused_user
done
