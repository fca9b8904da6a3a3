#!/usr/bin/env bash
# A/B of fused-news-kernel build variants (probe binaries nv_<name>_ns /
# nv_<name>), alternated on one box, f16x3 main pass only:
#   bash profiles/probes/ab_news.sh base variant ...
# (exit status 3 = the probe's cross-variant check, which has no f32 output
# to compare with here; any other failure ends the run)
set -uo pipefail
cd "$(dirname "$0")"
run() {
  NV_ONLY_H3=1 timeout -k 5 60 "$@" > /tmp/nv_run.txt 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then cat /tmp/nv_run.txt; echo "rc=$rc"; exit $rc; fi
}
for rep in 1 2 3; do
  for v in "$@"; do
    echo "== $v rep $rep"; run ./nv_${v}_ns 56320 10; grep "kernel avg" /tmp/nv_run.txt
  done
done
for v in "$@"; do echo "== $v stamps"; run ./nv_${v} 56320 3; grep -A4 "kernel avg" /tmp/nv_run.txt; done
