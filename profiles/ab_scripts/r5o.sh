#!/usr/bin/env bash
# r5o: cost of each gather-load group in the news kernel: probe builds without
# the Q (phase A), K (B epilogue) or V (phase C) prefetch loads, stamps per phase;
# also the FedAvg sync timing at world size 1 (RCCL and gloo)
set -uo pipefail
O=gpurun_out/r5o; mkdir -p $O
bash profiles/probes/ab_news.sh r5base r5noq r5nok r5nov > $O/news_loads_ab.txt 2>&1 || { tail -20 $O/news_loads_ab.txt; exit 1; }
cat $O/news_loads_ab.txt
for be in nccl gloo; do
  timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$([ $be = nccl ] && echo 1 || echo 2) profiles/fedavg_sync_bench.py --backend $be > $O/fedavg_$be.txt 2>&1 || { tail -20 $O/fedavg_$be.txt; exit 1; }
  grep '^{' $O/fedavg_$be.txt
done
