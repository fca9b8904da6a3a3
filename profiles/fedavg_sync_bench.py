"""FedAvg synchronisation cost on the GPU (BASELINE config 5, src/train.py:
the parameter all-reduce this build adds after the local steps).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29555 profiles/fedavg_sync_bench.py --backend nccl

Times train.FedAvg.sync (flatten the 21,955,400 parameters = 87.8 MB, one
all-reduce, divide by the world size, unflatten) and the all-reduce alone over
`--reps` calls with HIP events, at whatever world size it is launched with
(on one GPU: world size 1, the RCCL call path executed, no link traffic).
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    rank, local = int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if a.backend == "nccl" else {}
    dist.init_process_group(a.backend, **kw)
    import bench
    from newsrecommendationsystem_amd.distributed import all_reduce_
    from newsrecommendationsystem_amd.train import FedAvg
    model = bench.build_model(dev)
    fa = FedAvg(model, every=1)
    nbytes = fa.flat.numel() * 4

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / a.reps

    before = [p.detach().clone() for p in fa.params]
    sync_ms = timed(fa.sync)
    ar_ms = timed(lambda: all_reduce_(fa.flat))
    world = dist.get_world_size()
    same = all(torch.equal(p, b) for p, b in zip(fa.params, before)) if world == 1 else None
    out = {"backend": a.backend, "world": world, "param_bytes": nbytes, "reps": a.reps,
           "fedavg_sync_ms": round(sync_ms, 4), "all_reduce_ms": round(ar_ms, 4),
           "all_reduce_GBps_algbw": round(nbytes / (ar_ms / 1e3) / 1e9, 1),
           "world1_params_unchanged_bitwise": same,
           "note": "world size 1: the RCCL call path on one GPU (no xGMI traffic); the N > 1 cost is the "
                   "driver's 8-GPU run's to measure"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
