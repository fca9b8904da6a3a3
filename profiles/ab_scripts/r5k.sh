#!/usr/bin/env bash
# r5k: W-resident projection, A rows double-buffered in registers (a tile ahead): phase stamps + A/B against the streamed kernel
set -uo pipefail
O=gpurun_out/r5k; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_pxt.so timeout -k 10 120 python profiles/probes/px_wres_phases.py > $O/phases.txt 2>&1 || { cat $O/phases.txt; exit 1; }
cat $O/phases.txt
NRMS_LIB_PATH=_ab/lib_wres2.so bash _ab/ab_env.sh "NRMS_PROJ_WRES=0" "NRMS_PROJ_WRES=1" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
