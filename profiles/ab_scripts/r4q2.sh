#!/usr/bin/env bash
set -uo pipefail
mkdir -p gpurun_out/r4q2
bash profiles/probes/ab_news.sh r4final sched_ilp sched_iter sched_mem > gpurun_out/r4q2/sched.txt 2>&1; echo "rc=$?"
grep -E "==|kernel avg" gpurun_out/r4q2/sched.txt | paste - - | head -20
