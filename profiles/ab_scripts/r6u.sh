#!/usr/bin/env bash
# r6u: the news-kernel probe (profiles/probes/news_variants.hip: random ids,
# 56,320 titles, no dedupe) with the static group stride (HEAD~2's
# news_fused.hip, _ab/src/news_fused_static.hip) and the run-time claims,
# alternated on one box; then the projection's per-workgroup balance
set -uo pipefail
O=gpurun_out/r6u; mkdir -p $O
sed 's#../../newsrecommendationsystem_amd/csrc/news_fused.hip#news_fused_static.hip#' profiles/probes/news_variants.hip > _ab/src/nv_static.hip
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -I newsrecommendationsystem_amd/csrc -DNRMS_NO_STAMPS -mllvm -amdgpu-sched-strategy=max-ilp _ab/src/nv_static.hip -o /tmp/nv_static || exit 1
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -DNRMS_NO_STAMPS -mllvm -amdgpu-sched-strategy=max-ilp profiles/probes/news_variants.hip -o /tmp/nv_dyn || exit 1
for rep in 1 2 3; do
  for v in dyn static; do
    NV_ONLY_H3=1 timeout -k 10 120 /tmp/nv_$v 56320 10 > $O/nv_$v.txt 2>&1
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then cat $O/nv_$v.txt; exit $rc; fi
    echo "$v $(grep 'kernel avg' $O/nv_$v.txt)"
  done
done > $O/nv_ab.txt
cat $O/nv_ab.txt
NRMS_LIB_PATH=_ab/lib_pxt.so timeout -k 10 300 python profiles/probes/px_phases.py > $O/px_balance.txt 2>&1 || { tail -5 $O/px_balance.txt; exit 1; }
tail -3 $O/px_balance.txt
