#!/usr/bin/env bash
# Profile the bench workload on a GPU box (run from the repo root via gpurun):
#   bash profiles/run_profile.sh <tag>
# 1) kernel trace + stats (per-kernel durations), 2) FETCH_SIZE pass,
# 3) WRITE_SIZE pass (separate passes: TCC slots; never combined with
# sys/runtime traces). Outputs land in gpurun_out/prof_<tag>/.
set -euo pipefail
TAG=${1:-r01}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH=("$REPO/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras)
GATHER=("$REPO/profiles/kernel_driver.py" gather --iters 5)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" > "$OUT/bench_trace.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "${BENCH[@]}" > "$OUT/bench_fetch.json"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "${BENCH[@]}" > "$OUT/bench_write.json"
# the isolated gather (V = 1,048,576 table, config-2 shape) in the same three passes
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o gather -- python3 "${GATHER[@]}"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o gather -- python3 "${GATHER[@]}"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o gather -- python3 "${GATHER[@]}"
# SQ counters of every stage's kernel, from passes over the product path
# itself (nrms_forward on the bench batch): bench.py roofline.sq_counters
bash "$REPO/profiles/counters.sh" forward "$TAG"
find "$OUT" -name '*.csv' | sort
