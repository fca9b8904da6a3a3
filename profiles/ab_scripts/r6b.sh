#!/usr/bin/env bash
# r6b: projection read traffic: L2 hit / miss and EA read
# requests of every forward kernel (two counters per pass), then an A/B of the
# product library against the A rows loaded non-temporally (NRMS_PX_NT_A)
set -uo pipefail
O=gpurun_out/r6b; mkdir -p $O
REPO=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --list-avail > $REPO/$O/avail.txt 2>&1 ) || true
grep -o "TCC_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/tcc_names.txt || true
wc -l $O/tcc_names.txt
i=0
for pass in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_REQ_sum TCC_READ_sum"; do
  i=$((i + 1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $REPO/$O/tcc$i -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/tcc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/tcc$i.log; }
done
timeout -k 10 900 bash _ab/ab_bench.sh newsrecommendationsystem_amd/libnrms_hip.so _ab/lib_pxnta.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
