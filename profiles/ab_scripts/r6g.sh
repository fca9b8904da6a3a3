#!/usr/bin/env bash
# r6g: the profile recipe (kernel trace + stats, FETCH / WRITE passes, SQ
# passes of every stage) over the round-6 build checked by r6f
set -uo pipefail
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 1000 bash profiles/run_profile.sh r6g > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
