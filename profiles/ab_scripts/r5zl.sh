#!/usr/bin/env bash
# r5zl: error distribution vs the fp64 oracle per arithmetic (bench batch
# slice) for HEAD (rep's copies in one fma) and lib_norep (sequential adds)
set -uo pipefail
O=gpurun_out/r5zl; mkdir -p $O
for n in 128 512; do
  for lib in newsrecommendationsystem_amd/libnrms_hip.so _ab/lib_norep.so; do
    NRMS_LIB_PATH=$lib timeout -k 10 300 python -u tests/arith_err_probe.py $n 2>&1 | tee -a $O/err.txt || exit 1
  done
done
