#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4d; mkdir -p $O
bash profiles/probes/ab_news.sh base vperm adb w0e both qpre qpre_both > $O/news_ab.txt 2>&1 || exit 1
