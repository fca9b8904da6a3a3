#!/usr/bin/env bash
# r6d: where the projection's extra EA reads come from: L2 hit / miss and EA
# read requests of proj_qkv_kernel with its output stores predicated off
# (NRMS_PX_NOSTORE probe build; its outputs are not written, timing / counters only)
set -uo pipefail
O=gpurun_out/r6d; mkdir -p $O
REPO=$(pwd)
i=0
for pass in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_READ_sum TCC_WRITE_sum"; do
  i=$((i + 1))
  ( cd /tmp && export TMPDIR=/tmp && NRMS_LIB_PATH=$REPO/_ab/lib_pxnostore.so timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $REPO/$O/ns$i -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/ns$i.log 2>&1 || { echo "pass ns$i failed"; tail -5 $O/ns$i.log; }
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $REPO/$O/hd$i -o run -- python3 $REPO/profiles/kernel_driver.py forward --iters 5 ) > $O/hd$i.log 2>&1 || { echo "pass hd$i failed"; tail -5 $O/hd$i.log; }
done
ls $O
