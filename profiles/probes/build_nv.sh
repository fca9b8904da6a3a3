#!/usr/bin/env bash
# Build a fused-news probe variant pair: nv_<name> (phase stamps) and
# nv_<name>_ns (no stamps) with extra compile flags, for ab_news.sh.
#   bash profiles/probes/build_nv.sh <name> [-DFLAG ...]
set -euo pipefail
cd "$(dirname "$0")"
NAME=$1; shift
# (the product build uses the default scheduler for news_fused.hip; pass
# -mllvm -amdgpu-sched-strategy=... to try another)
CXX=(/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I ../../include "$@" news_variants.hip)
"${CXX[@]}" -o "nv_${NAME}" &
"${CXX[@]}" -DNRMS_NO_STAMPS -o "nv_${NAME}_ns" &
wait
