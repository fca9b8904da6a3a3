#!/usr/bin/env bash
# round-4 call c: news_fused memory-pipeline counters, probe by id range, quality settings
set -uo pipefail
O=gpurun_out/r4c; mkdir -p $O
bash profiles/mem_counters.sh news_fused r4c > $O/mem_counters.log 2>&1 || { echo mem_counters failed; exit 1; }
cd profiles/probes
for r in 70974 8192 512 1; do
  echo "== id_range $r" >> ../../$O/probe_idrange.txt
  NV_ONLY_H3=1 timeout -k 5 60 ./nv_base_ns 56320 10 $r >> ../../$O/probe_idrange.txt 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "rc=$rc" >> ../../$O/probe_idrange.txt; exit 1; fi
  NV_ONLY_H3=1 timeout -k 5 60 ./nv_base 56320 3 $r >> ../../$O/probe_idrange.txt 2>&1
  rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "rc=$rc" >> ../../$O/probe_idrange.txt; exit 1; fi
done
cd ../..
