#!/usr/bin/env bash
# r5g: kernel trace of 50 HIP training steps, HEAD vs deterministic kernels
set -uo pipefail
O=$PWD/gpurun_out/r5g; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for d in _ab/head .; do
  n=$(basename $d); [ "$n" = "." ] && n=cur
  (cd $R/$d && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 -m newsrecommendationsystem_amd.train --steps 50 --batch 64 > $O/prof_$n.log 2>&1) || { tail -5 $O/prof_$n.log; exit 1; }
  f=$(find $O/prof_$n -name "*kernel_stats.csv" | head -1); cp "$f" $O/train_kernel_stats_$n.csv
  echo "== $n"; head -22 $O/train_kernel_stats_$n.csv | cut -d, -f1-4 | cut -c1-150
done
rm -rf $O/prof_head $O/prof_cur
