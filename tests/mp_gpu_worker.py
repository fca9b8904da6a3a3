"""One rank of the multi-process GPU tests (tests/test_gpu_multiprocess.py):
started as a plain child process per rank (RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT in the environment), all ranks on cuda:0, collectives on gloo
(RCCL cannot put two ranks on one GPU). Writes its results as .npy / .json
files into the output directory given on the command line.

    python tests/mp_gpu_worker.py eval|fedavg|quality|collectives OUT_DIR [gloo|nccl]
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import weights as W  # noqa: E402


def _model(state, V, **cfg):
    from newsrecommendationsystem_amd import NRMS, NRMSConfig
    Cfg = type("Cfg", (NRMSConfig,), dict(num_words=V, **cfg))
    m = NRMS(Cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in state.items()})
    return m.to("cuda:0")


def run_eval(rank, world, out):
    """Config 4 semantics on the eval split: evaluate(process_group=...) over
    user shards vs the unsharded evaluate, and each shard's per-impression
    logits."""
    from newsrecommendationsystem_amd import data as Dt
    from newsrecommendationsystem_amd.distributed import shard_impressions
    from newsrecommendationsystem_amd.evaluate import EvalPlan, evaluate, score_plan
    g = np.load(os.path.join(ROOT, "tests", "golden", "nrms_flow_golden.npz"))
    d = os.path.join(ROOT, "tests", "golden", "flow", "eval")
    V = int(g["V_eval"])
    m = _model(W.nrms_state(int(g["seed"]), V), V).eval()
    sharded = evaluate(m, d, process_group=dist.group.WORLD)
    corpus = Dt.read_news_parsed(os.path.join(d, "news_parsed.tsv"))
    imps = Dt.read_behaviors(os.path.join(d, "behaviors.tsv"))
    mine = shard_impressions(imps, rank, world)
    scores, _ = score_plan(m, EvalPlan(corpus, mine))
    res = {"tuple": list(sharded), "ids": [im.impression_id for im in mine],
           "users": [im.user for im in mine]}
    np.save(os.path.join(out, f"rank{rank}_scores.npy"), scores.cpu().numpy())
    if rank == 0:
        res["unsharded"] = list(evaluate(m, d))
        full, _ = score_plan(m, EvalPlan(corpus, imps))
        np.save(os.path.join(out, "unsharded_scores.npy"), full.cpu().numpy())
        res["all_ids"] = [im.impression_id for im in imps]
        res["offsets"] = EvalPlan(corpus, imps).offsets.tolist()
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)


def run_fedavg(rank, world, out):
    """Config 5 on the HIP path: E local steps of the HIP training kernels +
    HipAdam on this rank's batches, then FedAvg's parameter all-reduce."""
    from newsrecommendationsystem_amd import train as TR
    V, B, E = 2000, 8, 3
    m = _model(W.nrms_state(77, V), V, dropout_probability=0.2).train()
    opt = TR.make_optimizer(m)
    fed = TR.FedAvg(m, every=E)
    batches = TR.synthetic_train_batches(100 + rank, E, B, V, device="cuda:0")
    losses, synced = [], []
    for cand, clk in batches:
        y = m.forward_ids(cand, clk)
        assert "NRMSTrain" in type(y.grad_fn).__name__, type(y.grad_fn)
        loss = TR.loss_fn(y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(float(loss.detach()))
        if fed.steps + 1 == E:   # the step that syncs: keep the local model first
            pre = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
            np.save(os.path.join(out, f"rank{rank}_pre.npy"), pre)
        synced.append(fed.step())
    post = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
    np.save(os.path.join(out, f"rank{rank}_post.npy"), post)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"losses": losses, "synced": synced, "optimizer": type(opt).__name__}, f)


def run_quality(rank, world, out):
    """Config 5 quality (newsrecommendationsystem_amd/quality.py): this rank is
    one FedAvg client on the HIP path (HIP training kernels + HipAdam, the
    parameter all-reduce of train.FedAvg over the process group), from the
    initialisation and batches the test wrote; rank 0 saves the result."""
    from newsrecommendationsystem_amd import quality as Q
    from newsrecommendationsystem_amd import train as TR
    from newsrecommendationsystem_amd.nrms import NRMS
    meta = json.load(open(os.path.join(out, "quality_meta.json")))
    cfg = Q.make_config(meta["V"], meta["lr"])
    m = NRMS(cfg)
    init = torch.load(os.path.join(out, "init.pt"), weights_only=True)
    m.load_state_dict(init)
    m = m.to("cuda:0")
    opt = TR.make_optimizer(m)
    fed = TR.FedAvg(m, every=meta["every"])
    b = np.load(os.path.join(out, f"batches{rank}.npz"))
    for k in range(b["cand"].shape[0]):
        cand = torch.from_numpy(b["cand"][k]).to("cuda:0")
        clk = torch.from_numpy(b["clk"][k]).to("cuda:0")
        TR.train_step(m, opt, cand, clk)
        fed.step()
    if rank == 0:
        torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, os.path.join(out, "hip_fedavg.pt"))
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"steps": int(b["cand"].shape[0]), "optimizer": type(opt).__name__}, f)


def run_collectives(rank, world, out):
    """The RCCL code paths of the product on a process group of this worker's
    backend (test_rccl_world1_collectives: "nccl" = RCCL, world size 1 on
    cuda:0, against the same calls on gloo): the bench's MAX timing
    all-reduce (fp64 GPU tensor) and stream-count SUM, evaluate()'s metric
    all-reduce over user shards, and FedAvg.sync of the HIP-trained
    parameters."""
    from newsrecommendationsystem_amd import train as TR
    from newsrecommendationsystem_amd.distributed import all_reduce_, max_over_ranks, sum_over_ranks
    from newsrecommendationsystem_amd.evaluate import evaluate
    dev = torch.device("cuda:0")
    res = {"backend": dist.get_backend()}
    res["max"] = max_over_ranks(1.25 + rank, dev)
    res["sum"] = sum_over_ranks(4096.0 * (rank + 1), dev)
    t = torch.arange(6, dtype=torch.float32, device=dev) * (rank + 1)
    res["all_reduce"] = all_reduce_(t).cpu().tolist()
    g = np.load(os.path.join(ROOT, "tests", "golden", "nrms_flow_golden.npz"))
    d = os.path.join(ROOT, "tests", "golden", "flow", "eval")
    V = int(g["V_eval"])
    m = _model(W.nrms_state(int(g["seed"]), V), V).eval()
    res["eval_group"] = list(evaluate(m, d, process_group=dist.group.WORLD))
    res["eval_plain"] = list(evaluate(m, d))
    V2, B = 2000, 8
    mt = _model(W.nrms_state(77, V2), V2, dropout_probability=0.2).train()
    opt = TR.make_optimizer(mt)
    fed = TR.FedAvg(mt, every=2)
    for cand, clk in TR.synthetic_train_batches(300 + rank, 2, B, V2, device="cuda:0"):
        TR.train_step(mt, opt, cand, clk)
        if fed.steps == 1:
            pre = torch.cat([p.detach().reshape(-1) for p in mt.parameters()]).cpu().numpy()
        res.setdefault("synced", []).append(fed.step())
    post = torch.cat([p.detach().reshape(-1) for p in mt.parameters()]).cpu().numpy()
    np.save(os.path.join(out, f"rank{rank}_pre.npy"), pre)
    np.save(os.path.join(out, f"rank{rank}_post.npy"), post)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)


def main():
    mode, out = sys.argv[1], sys.argv[2]
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    try:
        {"eval": run_eval, "fedavg": run_fedavg, "quality": run_quality,
         "collectives": run_collectives}[mode](rank, world, out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
