#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4e; mkdir -p $O
bash profiles/probes/ab_news.sh qpre qs1 qrot qrotw qs1rw qvp > $O/news_ab.txt 2>&1 || exit 1
bash _ab/ab_stage.sh _ab/lib_px8.so _ab/lib_px4.so _ab/lib_px4s.so > $O/proj_ab.txt 2>&1 || exit 1
NRMS_LIB_PATH=_ab/lib_px4s.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "qkv or forward or bench_batch" > $O/px4s_tests.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ -m gpu > $O/gputests.txt 2>&1 || exit 1
