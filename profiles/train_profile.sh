#!/usr/bin/env bash
# Kernel trace + stats of the HIP training step (batch 64, 50 steps):
#   bash profiles/train_profile.sh <tag>     (on a GPU box, from the repo root)
set -euo pipefail
TAG=${1:-train}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$REPO"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 -m newsrecommendationsystem_amd.train --batch 64 --steps 50 --warmup 5 > "$OUT/train.log" 2>&1
