#!/usr/bin/env bash
# r5e: deterministic training kernels -- GPU train tests, the RCCL/gloo
# collectives test (bitwise again), and training steps/s vs HEAD (x3 alternated)
set -uo pipefail
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_multiprocess.py -m gpu -k "train or rccl_world1_collectives or fedavg_hip" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.txt | tail -25
for rep in 1 2 3; do
  for d in _ab/head .; do
    (cd $d && timeout -k 10 120 python -m newsrecommendationsystem_amd.train --steps 200 --batch 64 2>&1 | tail -2 | sed "s|^|$d: |") >> $O/train_speed.txt || exit 1
  done
done
cat $O/train_speed.txt
