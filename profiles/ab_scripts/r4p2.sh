#!/usr/bin/env bash
set -uo pipefail
mkdir -p gpurun_out/r4final
bash profiles/probes/ab_news.sh r4final > gpurun_out/r4final/news_phases.txt 2>&1; echo "rc=$?"
cat gpurun_out/r4final/news_phases.txt | tail -12
