#!/usr/bin/env bash
# r5f: deterministic training kernels, two-pass column reductions -- train tests + speed vs HEAD
set -uo pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_multiprocess.py -m gpu -k "train or rccl_world1_collectives or fedavg_hip" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do
  for d in _ab/head .; do
    (cd $d && timeout -k 10 120 python -m newsrecommendationsystem_amd.train --steps 200 --batch 64 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$d', round(d['steps_per_s'],1), d['final_loss'])") >> $O/train_speed.txt || exit 1
  done
done
cat $O/train_speed.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -m newsrecommendationsystem_amd.train --steps 50 --batch 64 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/train_kernel_stats.csv; head -25 $O/train_kernel_stats.csv | cut -d, -f1-4
