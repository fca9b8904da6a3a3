#!/usr/bin/env bash
# r5n: stochastic PC sampling (beta) of the news kernel: per-instruction samples with stall reasons
set -uo pipefail
O=$PWD/gpurun_out/r5n; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d $O/pcs -o run -- python3 $R/profiles/kernel_driver.py news_fused --iters 5 > $O/pcs.log 2>&1
echo "rc=$?"
tail -20 $O/pcs.log
find $O/pcs -type f | head; for f in $(find $O/pcs -name "*.csv"); do echo "== $f"; head -3 $f; wc -l $f; done
