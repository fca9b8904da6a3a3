#!/usr/bin/env bash
# r5z: UserEncoder phase stamps (probe build lib_ut) on the bench's history distribution,
# the 512-thread chunked instance vs the 832-thread whole-tile instance
set -uo pipefail
O=gpurun_out/r5z; mkdir -p $O
for e in NRMS_USER_CHUNK=1 NRMS_USER_CHUNK=0; do
  echo "== $e" | tee -a $O/user_phases.txt
  env $e NRMS_LIB_PATH=_ab/lib_ut.so timeout -k 10 200 python profiles/probes/user_phases_padded.py 2>&1 | tee -a $O/user_phases.txt || exit 1
done
