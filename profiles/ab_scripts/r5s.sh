#!/usr/bin/env bash
# r5s: the projection with the item's tiles one after the other (lib_pxtile,
# NRMS_PX_TILE) against HEAD's library: its projection / forward tests, then
# bench stages alternated x2
set -uo pipefail
O=gpurun_out/r5s; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
NRMS_LIB_PATH=_ab/lib_pxtile.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "qkv or proj or forward or golden" > $O/pxtile_tests.log 2>&1 || { tail -30 $O/pxtile_tests.log; exit 1; }
tail -2 $O/pxtile_tests.log
timeout -k 10 600 bash _ab/ab_stage.sh $L _ab/lib_pxtile.so > $O/ab_stage.txt 2>&1 || { cat $O/ab_stage.txt; exit 1; }
cat $O/ab_stage.txt
