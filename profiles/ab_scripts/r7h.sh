#!/usr/bin/env bash
# r7h: what the Q|K|V weight packs cost inside forward_pack_kernel (the step's
# first launch): kernel trace of the product build against a probe build
# without them (results invalid, timing only)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
O=$REPO/gpurun_out/r7h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base nowp; do
  lib=$REPO/newsrecommendationsystem_amd/libnrms_hip.so
  [ $v = nowp ] && lib=$REPO/_ab/lib_nowp.so
  NRMS_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 $REPO/bench.py --no-cpu-baseline --no-extras --steps 20 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'pack' in r['Name'] or 'proj_qkv' in r['Name']: print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))
" "$f" $v
done
