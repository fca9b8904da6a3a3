#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4f; mkdir -p $O
bash profiles/probes/ab_news.sh qs1rw qs2 qs3 > $O/news_ab.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/gputests.txt 2>&1 || { tail -30 $O/gputests.txt; exit 1; }
tail -2 $O/gputests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['stages_ms'], d['roofline']['frac_vs_issued_peak'], d['fedavg_quality']['runs'][0]['auc_lift_hip'])"
