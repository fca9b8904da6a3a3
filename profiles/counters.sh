#!/usr/bin/env bash
# SQ counter passes for one stage: bash profiles/counters.sh <stage> <tag> [--unfused]
set -euo pipefail
STAGE=$1; TAG=$2; shift 2
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmc_${TAG}_${STAGE}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
DRV=("$REPO/profiles/kernel_driver.py" "$STAGE" --iters 5 "$@")
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/p1" -o run -- python3 "${DRV[@]}"
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d "$OUT/p2" -o run -- python3 "${DRV[@]}"
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL SQ_WAVES --output-format csv -d "$OUT/p3" -o run -- python3 "${DRV[@]}"
