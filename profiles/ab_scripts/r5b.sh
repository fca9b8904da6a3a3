#!/usr/bin/env bash
# r5b: where the news kernel's q|k|v gather is served from -- the same rows
# spread over 255 / 374 / 519 / 782 MB (NRMS_QKV_STRIDE, rows = 16 mod 128 B
# in every case), alternated x3 on one box; and the box's counter list.
set -uo pipefail
O=gpurun_out/r5b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
bash _ab/ab_env.sh "NRMS_QKV_STRIDE=900" "NRMS_QKV_STRIDE=1316" "NRMS_QKV_STRIDE=1828" "NRMS_QKV_STRIDE=2756" > $O/stride_ab.txt 2>&1 || { cat $O/stride_ab.txt; exit 1; }
cat $O/stride_ab.txt
