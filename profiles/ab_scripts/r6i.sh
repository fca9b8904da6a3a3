#!/usr/bin/env bash
# r6i: machine-scheduler / prefetch-depth sweep over the round-6 build: news
# kernel under the default and iterative-ILP schedulers (HEAD: max-ILP), the
# UserEncoder's W_add fragments 3 / 6 k-steps ahead (HEAD: 4); bench A/B x3
set -uo pipefail
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 1100 bash _ab/ab_bench.sh newsrecommendationsystem_amd/libnrms_hip.so _ab/lib_newsdef.so _ab/lib_newsiilp.so _ab/lib_userwd3.so _ab/lib_userwd6.so > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
