#!/usr/bin/env bash
# Memory-pipeline counter passes (TA / TD / TCP = vector L1, UTCL1 = L1 TLB) for
# one stage: bash profiles/mem_counters.sh <stage> <tag>. One pass per line:
# at most 2 TA, 2 TD, 4 TCP and 2 GRBM counters each (gfx950 slot limits).
set -euo pipefail
STAGE=$1; TAG=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/mem_${TAG}_${STAGE}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
DRV=("$REPO/profiles/kernel_driver.py" "$STAGE" --iters 5 "$@")
P=(
 "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
 "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_TOTAL_CYCLES_sum TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
 "TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_ACCESSES_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum"
)
i=0
for pass in "${P[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 "${DRV[@]}"
done
