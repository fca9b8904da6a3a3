#!/usr/bin/env bash
# r5fin3: the profile recipe (trace, traffic, SQ passes) over the final build
# (UserEncoder wave priority included), after r5fin2's suite / smoke / bench
set -uo pipefail
O=gpurun_out/r5fin3; mkdir -p $O
timeout -k 10 900 bash profiles/run_profile.sh r5fin3 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
