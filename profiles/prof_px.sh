#!/usr/bin/env bash
# Counter passes of the pre-split-W projection (proj_x6.hip) on the bench's
# vocabulary GEMM: bash profiles/prof_px.sh <tag> [stage]
set -euo pipefail
TAG=${1:-px}; STAGE=${2:-qkv_news}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
D=("$REPO/profiles/kernel_driver.py" "$STAGE")
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o a -- python3 "${D[@]}" --iters 5
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o a -- python3 "${D[@]}" --iters 3
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/h -o a -- python3 "${D[@]}" --iters 3
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/s1 -o a -- python3 "${D[@]}" --iters 3
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $OUT/s2 -o a -- python3 "${D[@]}" --iters 3
