#!/usr/bin/env bash
# r6c: UserEncoder head-split passes (round 6) against the round-5 chunked
# instance: bench A/B x3 alternated, then FETCH / WRITE passes of the forward
# with each library (traffic of fused_user_kernel per launch)
set -uo pipefail
O=gpurun_out/r6c; mkdir -p $O
REPO=$(pwd)
timeout -k 10 900 bash _ab/ab_bench.sh _ab/lib_user_r5.so newsrecommendationsystem_amd/libnrms_hip.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for lib in _ab/lib_user_r5.so newsrecommendationsystem_amd/libnrms_hip.so; do
  tag=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && NRMS_LIB_PATH=$REPO/$lib timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $REPO/$O/${tag}_$c -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/${tag}_$c.log 2>&1 || { echo "pmc $tag $c failed"; tail -5 $O/${tag}_$c.log; exit 1; }
    python profiles/pmc_sum.py $O/${tag}_$c fused_user
  done
done
