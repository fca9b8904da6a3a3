#!/usr/bin/env bash
# r5h: gemm_tn slice count (deterministic partials) -- training steps/s, HEAD vs 4096 / 8192 / 16384-block targets
set -uo pipefail
O=gpurun_out/r5h; mkdir -p $O
NRMS_LIB_PATH=_ab/lib_tn8192.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py -m gpu -k "deterministic or grads_match" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do
  for v in head tn4096 tn8192 tn16k; do
    if [ $v = head ]; then d=_ab/head; lib=$PWD/_ab/head/newsrecommendationsystem_amd/libnrms_hip.so; else d=.; lib=$PWD/_ab/lib_$v.so; fi
    (cd $d && NRMS_LIB_PATH=$lib timeout -k 10 120 python -m newsrecommendationsystem_amd.train --steps 300 --batch 64 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['steps_per_s'],1), d['final_loss'])") >> $O/train_speed.txt || exit 1
  done
done
cat $O/train_speed.txt
