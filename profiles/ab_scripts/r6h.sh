#!/usr/bin/env bash
# r6h: UserEncoder head split with 8, 9 or 10 first-pass heads (the first that
# adds no wave) against the round-5 task-index split: the user GPU tests, the
# bench logits bitwise, same-box A/B x3, FETCH / WRITE of fused_user_kernel
set -uo pipefail
O=gpurun_out/r6h; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "user" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
H=newsrecommendationsystem_amd/libnrms_hip.so
for lib in $H _ab/lib_user_r5.so; do
  tag=$(basename $lib .so)
  NRMS_LIB_PATH=$REPO/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --dump-logits $O/$tag > /dev/null 2> $O/$tag.err || { echo "dump $tag failed"; tail -5 $O/$tag.err; exit 1; }
done
python -c "
import numpy as np
a = np.load('$O/libnrms_hip.rank0.npz')['logits'].view(np.uint32); b = np.load('$O/lib_user_r5.rank0.npz')['logits'].view(np.uint32)
print('HEAD logits bitwise equal to the round-5 UserEncoder:', bool(np.array_equal(a, b)))"
timeout -k 10 900 bash _ab/ab_bench.sh $H _ab/lib_user_r5.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for lib in _ab/lib_user_r5.so $H; do
  tag=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && NRMS_LIB_PATH=$REPO/$lib timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $REPO/$O/${tag}_$c -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/${tag}_$c.log 2>&1 || { echo "pmc $tag $c failed"; tail -5 $O/${tag}_$c.log; exit 1; }
    python profiles/pmc_sum.py $O/${tag}_$c fused_user
  done
done
