"""Configs 4 and 5 with two processes on the GPU (world size 2, both ranks on
cuda:0, gloo collectives; the 8-GPU RCCL runs are the driver's): user-sharded
scoring (config 4) equals unsharded scoring, and FedAvg over the HIP training
kernels + HipAdam (config 5) leaves both ranks with the exact mean of the
local models. Each rank is a child process (tests/mp_gpu_worker.py)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mp_gpu_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(mode, out, world=2, timeout=240, backend="gloo"):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, mode, str(out), backend], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
            logs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, logs):
        assert p.returncode == 0, o[-3000:]
    return [json.load(open(os.path.join(out, f"rank{r}.json"))) for r in range(world)]


def test_user_sharded_evaluate_equals_unsharded(tmp_path):
    """evaluate(process_group=...) over 2 user shards == the unsharded tuple;
    every impression's logits from its shard == the unsharded logits bitwise;
    shards are disjoint, complete, and keep each user on one rank."""
    res = _run("eval", tmp_path)
    np.testing.assert_allclose(res[0]["tuple"], res[0]["unsharded"], rtol=1e-12, atol=0)
    assert res[0]["tuple"] == res[1]["tuple"]
    full = np.load(tmp_path / "unsharded_scores.npy")
    off = res[0]["offsets"]
    pos = {iid: k for k, iid in enumerate(res[0]["all_ids"])}
    seen = []
    owner = {}
    for r in range(2):
        sc = np.load(tmp_path / f"rank{r}_scores.npy")
        a = 0
        for iid, u in zip(res[r]["ids"], res[r]["users"]):
            k = pos[iid]
            n = off[k + 1] - off[k]
            assert np.array_equal(sc[a:a + n], full[off[k]:off[k + 1]]), iid
            a += n
            seen.append(iid)
            assert owner.setdefault(u, r) == r
        assert a == len(sc)
    assert sorted(seen) == sorted(res[0]["all_ids"]) and len(set(seen)) == len(seen)
    assert len(res[0]["ids"]) > 0 and len(res[1]["ids"]) > 0


def test_fedavg_hip_training_two_ranks(tmp_path):
    """Config 5: local HIP training steps (dropout 0.2) + HipAdam on each rank's
    batches, then FedAvg.sync: both ranks end bitwise identical, equal to the
    fp32 mean of the two local models."""
    res = _run("fedavg", tmp_path)
    assert all(r["optimizer"] == "HipAdam" for r in res)
    assert res[0]["synced"] == [False, False, True]
    pre = [np.load(tmp_path / f"rank{r}_pre.npy") for r in range(2)]
    post = [np.load(tmp_path / f"rank{r}_post.npy") for r in range(2)]
    assert not np.array_equal(pre[0], pre[1])          # the ranks trained apart
    assert np.array_equal(post[0], post[1])
    mean = (pre[0] + pre[1]) / np.float32(2)
    assert np.array_equal(post[0], mean.astype(np.float32))
    assert all(np.isfinite(r["losses"]).all() for r in res)


@pytest.mark.timeout(900)
def test_bench_two_ranks_stream_matches_one_rank(tmp_path):
    """The multi-rank bench path the driver's SCALE run takes (bench.py under
    torch.distributed.run, one process per rank, user-sharded config-4 stream;
    here gloo and both ranks on cuda:0): rc 0, exactly one JSON line (rank 0),
    the two shards together score every impression of the stream once, and
    every impression's logits equal the single-rank run's bitwise (the batch
    an impression lands in never changes its logits)."""
    n = 20000
    common = ["--stream", "--stream-impressions", str(n), "--no-extras", "--no-cpu-baseline", "--warmup", "1"]
    one = subprocess.run([sys.executable, "-u", "bench.py", *common, "--dump-logits", str(tmp_path / "one")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert one.returncode == 0, one.stderr[-3000:]
    port = _free_port()
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                          "--dist-backend", "gloo", *common, "--dump-logits", str(tmp_path / "two")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert two.returncode == 0, two.stderr[-3000:]
    lines = [ln for ln in two.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, two.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong" and rec["value"] > 0
    ref = np.load(tmp_path / "one.rank0.npz")
    assert np.array_equal(ref["idx"], np.arange(n))
    parts = [np.load(tmp_path / f"two.rank{r}.npz") for r in range(2)]
    idx = np.concatenate([p["idx"] for p in parts])
    assert len(idx) == n and np.array_equal(np.sort(idx), np.arange(n))
    assert len(set(parts[0]["idx"].tolist()) & set(parts[1]["idx"].tolist())) == 0
    logits = np.concatenate([p["logits"] for p in parts])
    assert np.isfinite(logits).all()
    assert np.array_equal(logits.view(np.uint32), ref["logits"][idx].view(np.uint32))


@pytest.mark.timeout(600)
def test_fedavg_training_quality_hip_vs_cpu(tmp_path):
    """Config 5's AUC half on a planted teacher (SURVEY §8d fallback; MIND is
    absent): two FedAvg clients on the HIP path (two processes on the GPU,
    HIP training kernels + HipAdam, train.FedAvg's all-reduce over gloo)
    against the same schedule on the CPU ATen path (train.py + torch Adam),
    from one initialisation, dropout 0; both evaluated with evaluate() on the
    teacher-labelled split: |AUC_hip - AUC_cpu| <= 0.002, and training moved
    the AUC away from the initial model's."""
    import torch
    from newsrecommendationsystem_amd import quality as Q
    steps, every, B = 32, 4, 16
    d = tmp_path / "split"
    cfg, teacher, corpus, titles, student = Q.setup(str(d))
    batches = [Q.teacher_batches(teacher, titles, 100 + 17 * r, steps, B) for r in range(2)]
    for r, bs in enumerate(batches):
        np.savez(tmp_path / f"batches{r}.npz", cand=np.stack([c.numpy() for c, _ in bs]),
                 clk=np.stack([k.numpy() for _, k in bs]))
    torch.save(student.state_dict(), tmp_path / "init.pt")
    with open(tmp_path / "quality_meta.json", "w") as f:
        json.dump({"V": cfg.num_words, "lr": cfg.learning_rate, "every": every}, f)
    res = _run("quality", tmp_path, timeout=400)
    assert all(r["optimizer"] == "HipAdam" and r["steps"] == steps for r in res)
    hip_sd = torch.load(tmp_path / "hip_fedavg.pt", weights_only=True)
    cpu_m, _, _ = Q.train_clients(student, batches, every, torch.device("cpu"))
    cpu_sd = {k: v.detach() for k, v in cpu_m.state_dict().items()}
    a_init = Q.auc_of(student.state_dict(), cfg, str(d))[0]
    a_hip = Q.auc_of(hip_sd, cfg, str(d))[0]
    a_cpu = Q.auc_of(cpu_sd, cfg, str(d))[0]
    assert abs(a_hip - a_cpu) <= 0.002, (a_hip, a_cpu)
    assert abs(a_hip - a_init) > 0.005, (a_init, a_hip)   # training moved it (0.574 -> 0.585 measured)
    for k in cpu_sd:
        if k.endswith("W_K.bias"):
            # its gradient is analytically zero (a key bias adds q . b_K to every
            # score of a query, which the normalisation divides out): Adam turns
            # the rounding noise of either path into +-lr steps, so the two
            # trajectories of this parameter are not comparable
            continue
        rel = float((hip_sd[k] - cpu_sd[k]).norm() / cpu_sd[k].norm().clamp_min(1e-30))
        assert rel < 1e-3, (k, rel)


@pytest.mark.timeout(600)
def test_rccl_world1_collectives(tmp_path):
    """Every RCCL call of the product, executed on the GPU: a world-size-1
    "nccl" process group on cuda:0 (init_process_group with device_id, as
    bench.py and distributed.init_from_env do) runs the bench's MAX timing
    all-reduce on an fp64 GPU tensor, its stream-count SUM, an fp32 tensor
    all-reduce, evaluate()'s metric all-reduce over the (single) user shard
    and FedAvg.sync of HIP-trained parameters; the same calls on gloo give
    the same results (world size 1: the identity, bitwise)."""
    outs = {}
    for be in ("nccl", "gloo"):
        d = tmp_path / be
        d.mkdir()
        outs[be] = _run("collectives", d, world=1, backend=be)[0]
        outs[be]["pre"] = np.load(d / "rank0_pre.npy")
        outs[be]["post"] = np.load(d / "rank0_post.npy")
    r, g = outs["nccl"], outs["gloo"]
    assert r["backend"] == "nccl" and g["backend"] == "gloo"
    assert r["max"] == g["max"] == 1.25 and r["sum"] == g["sum"] == 4096.0
    assert r["all_reduce"] == g["all_reduce"] == [float(i) for i in range(6)]
    assert r["eval_group"] == r["eval_plain"] == g["eval_group"]
    assert r["synced"] == g["synced"] == [False, True]
    for o in (r, g):   # the average over one client is the client's model, bitwise
        assert np.array_equal(o["post"], o["pre"])
    # same kernels and batches in two processes: the training kernels are
    # deterministic (no float atomics), so the trained and
    # synced parameters agree bitwise across the two backends
    assert np.array_equal(r["post"], g["post"])


def _shard_logits(rank, world, B):
    """The first B impressions of user shard rank/world scored in this process
    (no process group, eager nrms_forward, default arithmetic): the
    single-rank run of that shard."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from newsrecommendationsystem_amd import _native as N
    from newsrecommendationsystem_amd import stream as S
    from newsrecommendationsystem_amd.pipeline import TimedForward
    dev = torch.device("cuda:0")
    with N.gemm_arith(N.NRMS_GEMM_SPLIT_F16X3), torch.no_grad():
        model = bench.build_model(dev)
        idx = bench.stream_impressions(rank, world, B, dev)
        cand, clk = S.batch(0, idx, bench.V_WORDS)
        y = TimedForward(model, B, bench.C, bench.N_CLICKED, bench.L).run(cand, clk)
        torch.cuda.synchronize()
        return idx.cpu().numpy(), y.cpu().numpy()


def _check_weak_record(proc, n_gpus, backend):
    assert proc.returncode == 0, proc.stderr[-3000:]
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, proc.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n_gpus and rec["scaling"] == "weak" and rec["value"] > 0
    assert rec["graph_replay"] is True and "HIP graph" in rec["timed_path"]
    assert rec["process_group"] == backend and rec["forward_paths_bitwise_equal"] is True
    assert rec["config"]["global_batch"] == n_gpus * rec["config"]["impressions_per_gpu"]
    return rec


@pytest.mark.timeout(900)
def test_bench_two_ranks_weak_graph_gloo(tmp_path):
    """The driver's SCALE path (bench.py --gpus N without --stream: weak
    scaling, every rank captures its forward in a HIP graph and replays it
    under the process group; barrier + MAX timing) with two ranks sharing
    cuda:0 over gloo: rc 0, one JSON line, n_gpus 2, graph replay, and each
    rank's graph-replayed logits on its user shard bitwise equal to a
    single-rank run of that shard."""
    B = 1024
    port = _free_port()
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                          "--dist-backend", "gloo", "--steps", "5", "--warmup", "2", "--no-extras",
                          "--no-cpu-baseline", "--dump-logits", str(tmp_path / "two")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    _check_weak_record(two, 2, "gloo")
    seen = set()
    for r in range(2):
        got = np.load(tmp_path / f"two.rank{r}.npz")
        idx, ref = _shard_logits(r, 2, B)
        assert np.array_equal(got["idx"], idx) and len(idx) == B
        assert np.isfinite(ref).all()
        assert np.array_equal(got["logits"].view(np.uint32), ref.view(np.uint32)), r
        seen |= set(idx.tolist())
    assert len(seen) == 2 * B   # disjoint shards


@pytest.mark.timeout(900)
def test_bench_gpus2_self_launch_gloo(tmp_path):
    """The driver's plain form `python bench.py --gpus 2` with NO launcher
    around it: bench.py starts torch.distributed.run with two ranks as a child
    process itself (here gloo, both ranks on cuda:0) and relays rank 0's
    line: rc 0, one JSON line, n_gpus 2 = world_size, the FedAvg sync leg
    timed over the group, each rank's graph-replayed logits bitwise equal to
    `--as-shard r/2`'s single-process run of its shard."""
    B = 1024
    two = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--steps", "5",
                          "--warmup", "2", "--no-extras", "--no-cpu-baseline", "--dump-logits", str(tmp_path / "two")],
                         cwd=ROOT, capture_output=True, text=True, timeout=600,
                         env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    rec = _check_weak_record(two, 2, "gloo")
    assert rec["world_size"] == 2 and "child" in rec["launcher"]
    # stdout holds the JSON line and nothing else (gloo's notices go to stderr)
    assert len(two.stdout.strip().splitlines()) == 1, two.stdout[-2000:]
    fa = rec["fedavg_sync"]
    assert fa["world"] == 2 and fa["params"] == 21955400 and fa["fedavg_sync_ms"] > 0
    for r in range(2):
        shard = subprocess.run([sys.executable, "bench.py", "--as-shard", f"{r}/2", "--steps", "2", "--warmup", "1",
                                "--no-extras", "--no-cpu-baseline", "--dump-logits", str(tmp_path / f"s{r}")],
                               cwd=ROOT, capture_output=True, text=True, timeout=400)
        assert shard.returncode == 0, shard.stderr[-3000:]
        got, ref = np.load(tmp_path / f"two.rank{r}.npz"), np.load(tmp_path / f"s{r}.rank0.npz")
        assert len(got["idx"]) == B and np.array_equal(got["idx"], ref["idx"])
        assert np.array_equal(got["logits"].view(np.uint32), ref["logits"].view(np.uint32)), r


@pytest.mark.timeout(300)
def test_bench_gpus2_nccl_on_one_gpu_is_fatal():
    """`python bench.py --gpus 2` under nccl (RCCL) on a one-GPU box exits
    non-zero with a message instead of benchmarking one GPU."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-extras", "--no-cpu-baseline"],
                       cwd=ROOT, capture_output=True, text=True, timeout=200,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert p.returncode != 0 and "needs 2 GPUs" in p.stderr, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(600)
def test_bench_rccl_world1_weak_graph(tmp_path):
    """The same weak-scaling graph path on RCCL: torch.distributed.run with
    one process, backend "nccl" with device_id (--init-dist): the HIP graph
    captured and replayed with the RCCL communicator live, the RCCL barrier
    and MAX all-reduce around the timed region; one JSON line, logits equal
    to the single-rank run of shard 0/1 bitwise."""
    port = _free_port()
    one = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1",
                          "--init-dist", "--dist-backend", "nccl", "--steps", "5", "--warmup", "2",
                          "--no-extras", "--no-cpu-baseline", "--dump-logits", str(tmp_path / "rccl")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    rec = _check_weak_record(one, 1, "nccl")
    # config 5's collective timed on RCCL: at world size 1 the average of one
    # client is the client's own parameters, bitwise
    fa = rec["fedavg_sync"]
    assert fa["backend"] == "nccl" and fa["world"] == 1 and fa["params"] == 21955400
    assert fa["fedavg_sync_ms"] > 0 and fa["all_reduce_ms"] > 0
    assert fa["params_bitwise_unchanged_by_sync"] is True
    got = np.load(tmp_path / "rccl.rank0.npz")
    idx, ref = _shard_logits(0, 1, 1024)
    assert np.array_equal(got["idx"], idx)
    assert np.array_equal(got["logits"].view(np.uint32), ref.view(np.uint32))


@pytest.mark.timeout(600)
def test_bench_as_shard_equals_rank_shard(tmp_path):
    """bench.py --as-shard 1/2 (one process, no group) scores shard 1 of 2:
    the graph-replayed logits equal the in-process run of that shard."""
    one = subprocess.run([sys.executable, "-u", "bench.py", "--as-shard", "1/2", "--steps", "3", "--warmup", "1",
                          "--no-extras", "--no-cpu-baseline", "--dump-logits", str(tmp_path / "s")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert one.returncode == 0, one.stderr[-3000:]
    rec = json.loads([ln for ln in one.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["config"]["as_shard"] == "1/2" and rec["graph_replay"] is True and rec["n_gpus"] == 1
    got = np.load(tmp_path / "s.rank0.npz")
    idx, ref = _shard_logits(1, 2, 1024)
    assert np.array_equal(got["idx"], idx)
    assert np.array_equal(got["logits"].view(np.uint32), ref.view(np.uint32))


@pytest.mark.timeout(600)
def test_bench_rccl_world1(tmp_path):
    """bench.py's multi-rank path with RCCL, on one GPU: torch.distributed.run
    with one process, backend "nccl" (--init-dist takes the process-group
    branch at world size 1: init with device_id, barriers, the MAX timing
    all-reduce and the stream-count SUM); one JSON line, every impression of
    the sampled stream scored, logits equal to the run without a group."""
    n = 8192
    common = ["--stream", "--stream-impressions", str(n), "--no-extras", "--no-cpu-baseline", "--warmup", "1"]
    port = _free_port()
    one = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1",
                          "--init-dist", "--dist-backend", "nccl", *common,
                          "--dump-logits", str(tmp_path / "rccl")],
                         cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert one.returncode == 0, one.stderr[-3000:]
    lines = [ln for ln in one.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, one.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    plain = subprocess.run([sys.executable, "-u", "bench.py", *common, "--dump-logits", str(tmp_path / "plain")],
                           cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert plain.returncode == 0, plain.stderr[-3000:]
    a, b = np.load(tmp_path / "rccl.rank0.npz"), np.load(tmp_path / "plain.rank0.npz")
    assert np.array_equal(a["idx"], np.arange(n)) and np.array_equal(a["idx"], b["idx"])
    assert np.array_equal(a["logits"].view(np.uint32), b["logits"].view(np.uint32))
