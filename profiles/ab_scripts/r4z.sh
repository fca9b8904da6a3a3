#!/usr/bin/env bash
set -uo pipefail
O=gpurun_out/r4z; mkdir -p $O
for rep in 1 2 3; do
  for k in 1 2 3; do
    out=$(timeout -k 10 150 python bench.py --no-cpu-baseline --no-extras --steps 60 --inflight $k 2>>$O/err.txt) || { echo "fail k=$k"; tail -20 $O/err.txt; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['forward_paths_bitwise_equal'], d['config']['batches_in_flight'])" "$out" "$k" | tee -a $O/ab.txt
  done
done
