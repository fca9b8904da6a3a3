#!/usr/bin/env bash
# r5t: against HEAD's library, bench stages alternated x2 of
#   lib_pxtile  - projection, the item's tiles one after the other (NRMS_PX_TILE)
#   lib_uksplit - UserEncoder attention split by keys over lane pairs (NRMS_USER_KSPLIT)
#   lib_uk1024  - lib_uksplit with 1,024-thread workgroups for 33-50-title histories (NRMS_USER_NT50)
# after each variant's own GPU tests
set -uo pipefail
O=gpurun_out/r5t; mkdir -p $O
L=newsrecommendationsystem_amd/libnrms_hip.so
t() { NRMS_LIB_PATH=_ab/lib_$1.so timeout -k 10 400 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread -k "$3" > $O/$1_tests.log 2>&1 || { tail -30 $O/$1_tests.log; exit 1; }; echo "$1: $(tail -1 $O/$1_tests.log)"; }
t pxtile tests/test_gpu_parity.py "qkv or proj or forward_golden"
t uksplit tests/test_gpu_parity.py "user"
t uk1024 tests/test_gpu_parity.py "user"
timeout -k 10 600 bash _ab/ab_stage.sh $L _ab/lib_pxtile.so _ab/lib_uksplit.so _ab/lib_uk1024.so > $O/ab_stage.txt 2>&1 || { cat $O/ab_stage.txt; exit 1; }
cat $O/ab_stage.txt
