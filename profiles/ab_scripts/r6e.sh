#!/usr/bin/env bash
# r6e: (1) the UserEncoder head split (only where it adds no wave) and the
# embedding long-run path through their GPU tests; (2) same-box A/B x3 of HEAD
# against the round-5 UserEncoder and two projection probes (sc1 output
# stores, XCD-major item order); (3) every library's bench logits bitwise
# against HEAD's; (4) L2 / EA read counters of the sc1 probe's projection
set -uo pipefail
O=gpurun_out/r6e; mkdir -p $O
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -v -k "user or zipf or qkv_project" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
H=newsrecommendationsystem_amd/libnrms_hip.so
for lib in $H _ab/lib_user_r5.so _ab/lib_pxsc1.so _ab/lib_pxxcd.so; do
  tag=$(basename $lib .so)
  NRMS_LIB_PATH=$REPO/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --dump-logits $O/$tag > /dev/null 2> $O/$tag.err || { echo "dump $tag failed"; tail -5 $O/$tag.err; exit 1; }
done
python - <<PY
import numpy as np
h = np.load("$O/libnrms_hip.rank0.npz")["logits"].view(np.uint32)
for t in ("lib_user_r5", "lib_pxsc1", "lib_pxxcd"):
    print(t, "logits bitwise equal to HEAD:", bool(np.array_equal(np.load(f"$O/{t}.rank0.npz")["logits"].view(np.uint32), h)))
PY
timeout -k 10 1200 bash _ab/ab_bench.sh $H _ab/lib_user_r5.so _ab/lib_pxsc1.so _ab/lib_pxxcd.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
i=0
for pass in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i + 1))
  ( cd /tmp && export TMPDIR=/tmp && NRMS_LIB_PATH=$REPO/_ab/lib_pxsc1.so timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $REPO/$O/sc1_$i -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/sc1_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/sc1_$i.log; }
done
