#!/usr/bin/env bash
# A/B of fused-news-kernel build variants (probe binaries nv_<name>_ns /
# nv_<name>), alternated on one box: bash profiles/probes/ab_news.sh base bf32 ...
set -euo pipefail
cd "$(dirname "$0")"
for rep in 1 2 3; do
  for v in "$@"; do
    echo "== $v rep $rep"; timeout -k 5 60 ./nv_${v}_ns 56320 10 | grep "split-bf16"
  done
done
for v in "$@"; do echo "== $v stamps"; timeout -k 5 60 ./nv_${v} 56320 3 | grep -A4 "split-bf16"; done
