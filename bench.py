"""NRMS scoring throughput on MI355X (BASELINE.json metric / config 3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 1024] [--proj folded|direct|auto]

One step = one full NRMS forward (src/model/NRMS/__init__.py:19-48, eval
mode) over a batch of B synthetic MIND-shaped impressions resident in HBM:
1+K = 5 candidate titles and 50 clicked titles of 20 tokens each (history
left-padded with all-zero titles, src/dataset.py:79-83), V = 70,976 words,
d = 300, 15 heads, query dim 200 — every title is encoded (forward semantics).
The impressions come from the config-4 stream (newsrecommendationsystem_amd/
stream.py: 2,000,000 impressions over 1,000,000 users, sharded by
user_id % world): by default each rank scores the first B impressions of its
user shard every step (weak scaling, no data-path collective); with --stream
the ranks score the whole stream once (config 4, strong scaling). The time
is the max over ranks. Rank 0 prints one JSON line.

Extra fields: per-stage milliseconds (HIP events on the launch stream), the
roofline of the dominant kernel, and the CPU baseline (oracle ATen-order
restatement timed on this host, kind "port") with a parity check of the GPU
logits against it on the same sample.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "impressions/sec scored (NRMS, MIND-shape) at 1/2/4/8 MI355X; AUC vs CPU ref"
V_WORDS, D, L, C, N_CLICKED = 70976, 300, 20, 5, 50
PEAK_TFLOPS_F32 = 157.3   # MI355X fp32 MFMA/VALU dense peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0     # HBM3E spec peak


def synth_titles(gen, n, V, device):
    ids = torch.randint(1, V, (n, L), generator=gen, device=device)
    lens = torch.randint(5, L + 1, (n, 1), generator=gen, device=device)
    return torch.where(torch.arange(L, device=device)[None] < lens, ids, torch.zeros_like(ids))


def stream_impressions(rank, world, B, device, seed=0, n_impressions=None):
    """The first B impressions of this rank's user shard of the config-4
    stream (all of them when B is None), on the device."""
    from newsrecommendationsystem_amd import stream as S
    idx = S.shard(seed, rank, world, n_impressions or S.N_IMPRESSIONS, S.N_USERS, device)
    return idx if B is None else idx[:B]


def synth_impressions(seed, B, V, device):
    """SURVEY §8d synthetic inputs: candidates [B,C,L], clicked [B,N,L]."""
    gen = torch.Generator(device=device).manual_seed(seed)
    cand = synth_titles(gen, B * C, V, device).view(B, C, L)
    clk = synth_titles(gen, B * N_CLICKED, V, device).view(B, N_CLICKED, L)
    hist = torch.randint(1, N_CLICKED + 1, (B, 1), generator=gen, device=device)
    pad = torch.arange(N_CLICKED, device=device)[None] < (N_CLICKED - hist)
    clk = torch.where(pad[:, :, None], torch.zeros_like(clk), clk)
    return cand.contiguous(), clk.contiguous()


def build_model(device, seed=0):
    from newsrecommendationsystem_amd import NRMS, NRMSConfig

    class Cfg(NRMSConfig):
        hip_check_ids = False   # inputs are generated in range on the device

    torch.manual_seed(seed)
    emb = torch.randn(V_WORDS, D)  # N(0,1), row 0 not zeroed (data_preprocess.py:272-277)
    return NRMS(Cfg, emb).to(device).eval()


def load_traffic(kernel):
    """Per-launch HBM bytes of `kernel` from the committed PMC summary (rocprofv3
    --pmc FETCH_SIZE / WRITE_SIZE, gfx950-corrected), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_ranges(cpus):
    """'0-15,64-79' style summary of a CPU set."""
    cpus, out, a = sorted(cpus), [], None
    for i, c in enumerate(cpus):
        if a is None:
            a = c
        if i + 1 == len(cpus) or cpus[i + 1] != c + 1:
            out.append(f"{a}-{c}" if c != a else f"{a}")
            a = None
    return ",".join(out)


def cpu_baseline(model, cand, clk, reps=5):
    """SURVEY §8d CPU leg: the oracle's ATen-order restatement of the
    reference forward (oracle/nrms_torch_cpu.py, bit-exact with the reference
    on the golden vectors) on the SAME batch as the GPU step (B impressions),
    median of `reps` timed runs after one warm-up, on this process's CPU
    share (OMP_NUM_THREADS / affinity; the affinity set is recorded: the
    host's other tenants move single runs by up to ~35 %, so the spread of
    the runs is reported beside the median); also the GPU-vs-CPU logits
    parity on that batch."""
    from oracle import nrms_torch_cpu as T
    threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    cand_c, clk_c = cand.cpu(), clk.cpu()
    times = []
    try:
        with torch.no_grad():
            ref = T.forward(cand_c, clk_c, sd)   # warm
            for _ in range(reps):
                t0 = time.perf_counter()
                ref = T.forward(cand_c, clk_c, sd)
                times.append(time.perf_counter() - t0)
            gpu = model.forward_ids(cand, clk).cpu()
    finally:
        torch.set_num_threads(prev)
    B = cand.shape[0]
    med = sorted(times)[len(times) // 2]
    err = float(((gpu - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-30)).max())
    aff = os.sched_getaffinity(0)
    info = {"value": round(B / med, 2), "unit": "impressions/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "affinity": _cpu_ranges(aff), "affinity_cpus": len(aff),
            "runs_s": [round(t, 3) for t in times],
            "spread": round((max(times) - min(times)) / med, 3),
            "sample": f"NRMS.forward over the bench batch ({B} impressions, 1+K=5, 50 clicked, L=20, "
                      f"V={V_WORDS}) via oracle/nrms_torch_cpu.py, torch {torch.__version__}, "
                      f"{threads} threads, median of {reps} runs "
                      f"({', '.join(f'{t:.2f}' for t in times)} s)"}
    parity = {"sample_impressions": B, "max_normwise_rel_err_logits": err,
              "tolerance": 1e-3, "ok": bool(err <= 1e-3)}
    return info, parity, ref


def eval_auc_check(model, device, n_impressions=4000, seed=11):
    """The metric's second half, "AUC vs CPU ref": a synthetic MIND-shaped split
    (reference file formats) whose labels are drawn from this model's own
    logits (planted teacher, temperature 1), scored by the GPU eval pipeline
    (newsrecommendationsystem_amd.evaluate) and by the CPU restatement of
    src/evaluate.py (oracle/eval_oracle.py, the cpu_baseline leg)."""
    import tempfile
    import numpy as np
    from newsrecommendationsystem_amd import data as Dt
    from newsrecommendationsystem_amd.evaluate import EvalPlan, evaluate, score_plan
    from oracle import eval_oracle as EO

    def teacher(corpus, imps):
        scores, _ = score_plan(model, EvalPlan(corpus, imps))
        sc = scores.cpu().numpy()
        plan = EvalPlan(corpus, imps)
        return [sc[a:b] for a, b in zip(plan.offsets[:-1], plan.offsets[1:])]

    with tempfile.TemporaryDirectory() as d:
        corpus, imps = Dt.synthetic_split(d, seed=seed, n_news=6000, n_users=1500,
                                          n_impressions=n_impressions, V=V_WORDS, teacher=teacher)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gpu = evaluate(model, d)
        torch.cuda.synchronize()
        t_gpu = time.perf_counter() - t0
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    t0 = time.perf_counter()
    cpu, _, _ = EO.evaluate(sd, corpus, imps)
    t_cpu = time.perf_counter() - t0
    return {"impressions": n_impressions, "auc_gpu": gpu[0], "auc_cpu": cpu[0],
            "abs_diff_auc": abs(gpu[0] - cpu[0]), "tolerance": 0.002,
            "mrr_gpu": gpu[1], "mrr_cpu": cpu[1], "ndcg10_gpu": gpu[3], "ndcg10_cpu": cpu[3],
            "eval_wall_s_gpu_incl_file_io": round(t_gpu, 3), "eval_wall_s_cpu": round(t_cpu, 3),
            "labels": "planted teacher (Bernoulli(sigmoid(model logit)))"}


def eval_throughput(model, device, seed=5):
    """evaluate() impressions/s on a synthetic split of MIND-small-dev's shape
    (73,152 impressions, 42,416 news, 50,000 users, U{2..73} candidates per
    impression; uniform p = 0.2 labels), the host stages (reading the two TSV
    files, building the EvalPlan) timed apart from the GPU passes (news
    vectors, user vectors, the score_pairs and impression_metrics launches,
    the nanmean) -- src/evaluate.py:171-272's whole job."""
    import tempfile
    from newsrecommendationsystem_amd import data as Dt
    from newsrecommendationsystem_amd import evaluate as EV
    shape = dict(n_news=42416, n_users=50000, n_impressions=73152, V=V_WORDS, min_cands=2, max_cands=73)

    def clock():
        torch.cuda.synchronize(device)
        return time.perf_counter()

    with tempfile.TemporaryDirectory() as d:
        Dt.synthetic_split(d, seed=seed, **shape)
        t0 = clock()
        # the readers evaluate() uses (native for the MIND form: csrc/tsv_io.hip)
        corpus = Dt.read_news_parsed(os.path.join(d, "news_parsed.tsv"))
        imps = Dt.load_behaviors(os.path.join(d, "behaviors.tsv"))
        t1 = clock()
        plan = EV.EvalPlan(corpus, imps, num_clicked=model.config.num_clicked_news_a_user)
        t2 = clock()
        with torch.no_grad():
            tab = EV.news_vectors(model, plan.corpus.titles)
            t3 = clock()
            users = EV.user_vectors(model, tab, plan.hist_rows)
            t4 = clock()
            del tab, users
            _, metrics = EV.score_plan(model, plan)   # (all passes again, for the total)
            means = EV.reduce_means(*EV.nan_sums(metrics))
        t5 = clock()
        t_e0 = clock()
        again = EV.evaluate(model, d)
        t_e1 = clock()
    n = plan.n_impressions
    return {
        "workload": "synthetic split of MIND-small-dev shape: 73,152 impressions, 42,416 news, "
                    "50,000 users, U{2..73} candidates, U{0..70} clicked (first 50 kept)",
        "impressions": n, "candidates": int(plan.cand.shape[0]), "distinct_histories": int(plan.hist_rows.shape[0]),
        "host_read_s": round(t1 - t0, 3), "host_plan_s": round(t2 - t1, 3),
        "host_reader": type(imps).__name__,
        "gpu_news_vectors_s": round(t3 - t2, 4), "gpu_user_vectors_s": round(t4 - t3, 4),
        "gpu_all_passes_s": round(t5 - t4, 4),
        "gpu_impressions_per_s": round(n / (t5 - t4), 1),
        "evaluate_wall_s": round(t_e1 - t_e0, 3),
        "evaluate_impressions_per_s": round(n / (t_e1 - t_e0), 1),
        "auc": means[0], "evaluate_equal_to_stagewise": bool(tuple(again) == tuple(means)),
        "note": "evaluate() = read + plan + all GPU passes (its own clock); gpu_all_passes_s = "
                "news vectors + user vectors + score_pairs + impression_metrics + nanmean"}


def _time_launches(fn, reps, device):
    """Average ms of fn() over reps launches, HIP events on the launch stream."""
    s = torch.cuda.current_stream(device)
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


GEMM_CODES = {"f16x3": 2, "x6": 0, "f32": 1}   # nrms_gemm_arith_t


def gemm_legs(model, cand, clk, mode, device, base, y_base):
    """The timed step (nrms_forward, graph-replayed like the headline) under
    the other GEMM arithmetics:
    ms / step, impressions / s, and the logits' distance to the default's
    (the CPU-port distance is added after the cpu_baseline leg)."""
    from newsrecommendationsystem_amd import _native as Nat
    from newsrecommendationsystem_amd.pipeline import TimedForward
    lib = Nat.load()
    B = cand.shape[0]
    legs = {}
    for g in ("x6", "f32"):
        if g == base:
            continue
        prev = lib.nrms_set_gemm_arith(GEMM_CODES[g])
        try:
            f = TimedForward(model, B, C, N_CLICKED, L, proj_mode=mode)
            with torch.no_grad():
                y = f.run(cand, clk).clone()
                eager = _time_launches(lambda: f.run(cand, clk), 10, device)
                # the arithmetic switch is read at enqueue time: the captured
                # graph replays this leg's kernels
                gr = capture_graph(f, cand, clk, device)
                f.logits.fill_(float("nan"))
                gr.replay()
                same = bool(torch.equal(f.logits, y))
                ms = _time_launches(gr.replay, 20, device)
        finally:
            lib.nrms_set_gemm_arith(prev)
        legs[g] = {"ms_per_step": round(ms, 4), "impressions_per_s": round(B / (ms / 1e3), 1),
                   "eager_ms_per_step": round(eager, 4), "graph_logits_equal_eager": same,
                   "max_normwise_rel_err_vs_default": float(
                       ((y - y_base).norm(dim=1) / y_base.norm(dim=1).clamp_min(1e-30)).max()),
                   "timing": "nrms_forward captured in a HIP graph and replayed (as the headline), HIP "
                             "events over 20 replays; eager: 10 Python-issued calls",
                   "_logits": y}
        del gr, f
    return legs


def capture_graph(f, cand, clk, device):
    """f.run(cand, clk) captured into a HIP graph (one warm call on a side
    stream first, as torch.cuda.graph requires)."""
    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        f.run(cand, clk)
    torch.cuda.current_stream(device).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        f.run(cand, clk)
    return g


def gather_hbm(device, V=1 << 20, n_titles=100_000, reps=20):
    """SURVEY §8d gather figure: nrms_embedding_gather alone over a 1.26 GB
    table (V = 1,048,576, beyond the 256 MB Infinity Cache), config-2 shape
    (100k titles x 20 tokens). Algorithmic bytes per token: 8 (id) + 1200
    (row read) + 1200 (row write)."""
    from newsrecommendationsystem_amd import _native as Nat
    gen = torch.Generator(device=device).manual_seed(5)
    table = torch.randn(V, D, generator=gen, device=device)
    ids = synth_titles(gen, n_titles, V, device).reshape(-1).contiguous()
    out = torch.empty(ids.numel(), D, device=device)
    st = Nat.stream_handle(device)
    fn = lambda: Nat.call("nrms_embedding_gather", Nat.ptr(ids), ids.numel(), Nat.ptr(table), V, D,
                          Nat.ptr(out), st)
    ms = _time_launches(fn, reps, device)
    ok = bool(torch.equal(out[:4096], table[ids[:4096]]))   # bit-exact spot check
    nbytes = ids.numel() * (8 + 2 * 4 * D)
    gbs = nbytes / (ms / 1e3) / 1e9
    del table, out
    traffic = load_traffic("gather")
    out = {"kernel": "gather_rows_kernel", "workload": f"{n_titles} titles x {L} tokens, V={V}, D={D}",
           "bound": "hbm", "ms": round(ms, 4), "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
           "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": nbytes,
           "traffic": traffic, "bit_exact_sample": ok}
    if traffic:
        # on the bytes that reached HBM (PMC): the padding rows (id 0) are served on-die
        tgbs = traffic / (ms / 1e3) / 1e9
        out["traffic_achieved"] = round(tgbs, 1)
        out["frac_on_traffic"] = round(tgbs / PEAK_HBM_GBS, 4)
    return out


def news_encoder_cfg2(model, device, n_titles=100_000, reps=10):
    """BASELINE config 2: NewsEncoder-only forward (get_news_vector) on 100k
    synthetic titles; the folded Q|K|V vocabulary projection is recomputed on
    every call (cache off), so each call does all of the encoder's work."""
    gen = torch.Generator(device=device).manual_seed(6)
    titles = synth_titles(gen, n_titles, V_WORDS, device)
    from newsrecommendationsystem_amd import _native as Nat
    cfg = model.news_encoder.config
    saved = (cfg.hip_cache_folded_table, cfg.hip_proj_mode)
    cfg.hip_cache_folded_table, cfg.hip_proj_mode = False, Nat.NRMS_PROJ_FOLDED
    try:
        with torch.no_grad():
            ms = _time_launches(lambda: model.get_news_vector({"title": titles}), reps, device)
    finally:
        cfg.hip_cache_folded_table, cfg.hip_proj_mode = saved
    return {"workload": f"BASELINE cfg2: NewsEncoder forward, {n_titles} titles x {L} tokens, "
                        f"V={V_WORDS}, projection folded per call", "ms_per_call": round(ms, 4),
            "titles_per_s": round(n_titles / (ms / 1e3), 1)}


PEAK_TFLOPS_BF16 = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def load_sq(kernel):
    """MFMA-busy fraction and VALU:MFMA ratio of `kernel` from the committed
    SQ counter passes (profiles/sq_counters.json, made by profiles/sq_summary.py
    from rocprofv3 --pmc runs), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "sq_counters.json")) as f:
            return json.load(f).get(kernel)
    except (OSError, ValueError):
        return None


# 16-bit products per fp32 product of each split arithmetic, per GEMM kind:
# the Q|K|V projections (f16x3: 3 products; 4 only for weight sets with a
# column that fits in 11 bits, not the bench's random weights), the additive
# GEMMs (f16x3: 2 x 2 planes -> 3 products); x6: 6 everywhere
PRODUCTS = {"f16x3": {"proj": 3, "additive": 3}, "x6": {"proj": 6, "additive": 6}, "f32": None}


def issue_floor_ms(stage, w, gemm):
    """Time a stage's matrix / vector instructions need at the MI355X peaks
    with nothing else in the way (the stage's FLOP split): split GEMMs issue
    their 16-bit products at 2.5 PF dense, exact f32 MFMA, the attention
    contractions and the pooling run at 157.3 TF (f32 MFMA = the vector rate);
    the scorer is bound by its HBM bytes at 8 TB/s."""
    if stage == "score":
        return w["bytes"] / (PEAK_HBM_GBS * 1e9) * 1e3
    f = w.get("split")
    if f is None:
        return None
    prod = PRODUCTS[gemm]
    kind = "proj" if stage.startswith("qkv") else "additive"
    gemm_s = (f["gemm"] * prod[kind] / (PEAK_TFLOPS_BF16 * 1e12) if prod
              else f["gemm"] / (PEAK_TFLOPS_F32 * 1e12))
    rest_s = (f.get("attention", 0) + f.get("pool", 0)) / (PEAK_TFLOPS_F32 * 1e12)
    return (gemm_s + rest_s) * 1e3


def bytes_floor_ms(w):
    """Time a stage's algorithmic bytes (what it must read and write,
    pipeline.ForwardPlan.work) take at the 8 TB/s HBM peak."""
    return w["bytes"] / (PEAK_HBM_GBS * 1e9) * 1e3


def n_all_titles(B):
    return B * (C + N_CLICKED)


def run_steps(fwd, batches, steps, events=None):
    for k in range(steps):
        cand, clk = batches[k % len(batches)]
        fwd.run(cand, clk, events[k] if events else None)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, backend):
    """`python bench.py --gpus N` (N > 1) started without a launcher: run
    torch.distributed.run with N processes (one per GPU) as a CHILD process
    -- before this process has touched the GPU, and never by exec -- whose
    rank 0 prints the JSON line straight to our stdout; return its exit code.
    With the nccl (RCCL) backend every rank needs its own GPU: fewer visible
    devices than N is fatal (gloo may share one GPU, for rehearsals)."""
    import subprocess
    if backend == "nccl":
        have = torch.cuda.device_count()   # counts devices without initialising HIP
        if have < n:
            print(f"bench.py: --gpus {n} with the nccl backend needs {n} GPUs, {have} visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, NRMS_BENCH_LAUNCHER="bench.py --gpus (torch.distributed.run child)")
    # relay rank 0's JSON line alone to stdout; anything else the ranks print
    # there (gloo's connection notices, from its C++ side) goes to stderr
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        at = line.find('{"metric"')
        if at >= 0:
            sys.stdout.write(line[at:])
            sys.stdout.flush()
            if at > 0:
                sys.stderr.write(line[:at] + "\n")
        else:
            sys.stderr.write(line)
    return p.wait()


def fedavg_sync_leg(model, device, dist, reps=5):
    """Config 5's collective, timed once the scoring steps are done: one
    train.FedAvg sync of all 21,955,400 parameters (flatten, all-reduce over
    the process group -- RCCL over xGMI under nccl --, divide by the world
    size, unflatten; the insertion point after src/train.py:233) and the
    all-reduce alone, HIP events over `reps` calls after a warm one, max over
    ranks. The parameters are restored afterwards (the ranks hold the same
    weights, but a ring sum of W equal values need not round back to them)."""
    from newsrecommendationsystem_amd.distributed import all_reduce_, max_over_ranks
    from newsrecommendationsystem_amd.train import FedAvg
    fa = FedAvg(model, every=1)
    before = [p.detach().clone() for p in fa.params]
    world = dist.get_world_size()
    nbytes = fa.flat.numel() * 4

    def timed(fn):
        fn()
        torch.cuda.synchronize(device)
        dist.barrier()
        s = torch.cuda.current_stream(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        e1.synchronize()
        return max_over_ranks(e0.elapsed_time(e1) / reps, device)

    with torch.no_grad():
        sync_ms = timed(fa.sync)
        identity = all(torch.equal(p, b) for p, b in zip(fa.params, before))
        ar_ms = timed(lambda: all_reduce_(fa.flat))
        for p, b in zip(fa.params, before):
            p.copy_(b)
    algbw = nbytes / (ar_ms / 1e3) / 1e9
    return {"params": fa.flat.numel(), "param_bytes": nbytes, "world": world, "backend": dist.get_backend(),
            "reps": reps, "fedavg_sync_ms": round(sync_ms, 4), "all_reduce_ms": round(ar_ms, 4),
            "all_reduce_algbw_GBps": round(algbw, 1),
            "all_reduce_busbw_GBps": round(algbw * 2 * (world - 1) / world, 1),
            "params_bitwise_unchanged_by_sync": identity,
            "note": "train.FedAvg.sync (flatten + all_reduce + divide + unflatten) and the all-reduce alone, "
                    "after the timed region; busbw = algbw * 2(W-1)/W (ring all-reduce); parameters restored "
                    "after the measurement"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 50; with --stream: every batch of the shard)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024, help="impressions per GPU per step")
    ap.add_argument("--proj", choices=["folded", "direct", "auto"], default="folded")
    ap.add_argument("--stream", action="store_true",
                    help="BASELINE cfg4: score the whole user-sharded 2M-impression stream once "
                         "(strong scaling; --steps is then the number of batches, 0 = all)")
    ap.add_argument("--stream-impressions", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU-port leg (and the CPU-side AUC check and the FedAvg quality run)")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the reference-scale FedAvg quality run (quality.run_scaled, ~20 s)")
    ap.add_argument("--as-shard", default=None, metavar="R/W",
                    help="without a process group, take rank R of W's user shard of the stream (tests: a "
                         "single-rank run of one shard of a multi-rank job)")
    ap.add_argument("--unfused", action="store_true", help="separate MHSA / additive / pool kernels")
    ap.add_argument("--no-extras", action="store_true", help="skip the gather / config-2 / direct figures")
    ap.add_argument("--no-graph", action="store_true", help="time the eager call loop instead of a HIP graph replay")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight: that many captured forwards (own workspace, logits and stream) "
                         "replayed in turn, so one batch's launch boundaries and kernel tails overlap "
                         "another's kernels (graph path only)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="process-group backend for the barrier / max-over-ranks timing (nccl = RCCL); "
                         "gloo lets several ranks share one GPU for a rehearsal")
    ap.add_argument("--init-dist", action="store_true",
                    help="initialise the process group (and take the barrier / max-over-ranks path) even "
                         "at world size 1: the RCCL code path on one GPU (tests)")
    ap.add_argument("--dump-logits", default=None, metavar="PATH",
                    help="after the timed region, score every batch once more and save this rank's "
                         "impression indices and logits to PATH.rank<r>.npz (multi-rank tests)")
    ap.add_argument("--gemm", choices=["f16x3", "x6", "f32"], default="f16x3",
                    help="GEMM arithmetic: split-f16 news additive GEMM and Q|K|V projections "
                         "(default), split-bf16 x6 everywhere, or exact f32 MFMA (all fp32-accurate)")
    args = ap.parse_args()
    if args.no_cpu_baseline:
        args.no_quality = True

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start one (a child, before any GPU call)
        sys.exit(launch_ranks(args.gpus, args.dist_backend))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus={args.gpus}: the launcher's process "
                         f"count and --gpus must agree")
    if world > 1 and args.dist_backend == "nccl" and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks on the nccl backend need {world} GPUs, "
                         f"{torch.cuda.device_count()} visible")
    device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(device)
    dist = None
    if world > 1 or args.init_dist:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)

    from newsrecommendationsystem_amd import _native as Nat
    from newsrecommendationsystem_amd import stream as S
    from newsrecommendationsystem_amd.pipeline import ForwardPlan, TimedForward

    Nat.load().nrms_set_gemm_arith({"f16x3": Nat.NRMS_GEMM_SPLIT_F16X3, "x6": Nat.NRMS_GEMM_SPLIT_BF16X6,
                                    "f32": Nat.NRMS_GEMM_F32}[args.gemm])
    mode = {"folded": Nat.NRMS_PROJ_FOLDED, "direct": Nat.NRMS_PROJ_DIRECT, "auto": Nat.NRMS_PROJ_AUTO}[args.proj]
    model = build_model(device)
    B = args.batch
    # this rank's user shard of the config-4 stream (user_id % world); inputs
    # are generated into HBM before the timed region
    s_rank, s_world = rank, world
    if args.as_shard:
        if dist:
            raise SystemExit("--as-shard is for single-process runs")
        s_rank, s_world = (int(x) for x in args.as_shard.split("/"))
    idx = stream_impressions(s_rank, s_world, None if args.stream else B, device,
                             n_impressions=args.stream_impressions)
    if args.stream:
        batches = [S.batch(0, idx[a:a + B], V_WORDS) for a in range(0, idx.numel(), B)]
    else:
        batches = [S.batch(0, idx, V_WORDS)]
    full = [b for b in batches if b[0].shape[0] == B]
    tail = [b for b in batches if b[0].shape[0] != B]
    # the timed step is the product path itself (nrms_forward, stage events
    # inside the library); ForwardPlan (the stage ABI, one call per stage)
    # gives the per-stage algorithmic work and the --unfused stage kernels
    plan = ForwardPlan(model, B, C, N_CLICKED, L, proj_mode=mode, fused=not args.unfused)
    fwd = plan if args.unfused else TimedForward(model, B, C, N_CLICKED, L, proj_mode=mode)
    tail_fwd = None
    if tail:
        Bt = tail[0][0].shape[0]
        tail_fwd = (ForwardPlan(model, Bt, C, N_CLICKED, L, proj_mode=mode, fused=False) if args.unfused
                    else TimedForward(model, Bt, C, N_CLICKED, L, proj_mode=mode))
    stages = fwd.stages
    n_st = len(stages)
    steps = 50 if args.steps is None else args.steps
    if args.stream:
        steps = len(full) if not args.steps or args.steps > len(full) else args.steps
    cand, clk = full[0]

    with torch.no_grad():
        run_steps(fwd, full, args.warmup)
        if tail_fwd is not None:
            tail_fwd.run(*tail[0])
        # one un-timed check: the timed path, the module's forward and the
        # stage-by-stage plan give bitwise the same logits
        y_fwd = fwd.run(cand, clk).clone()
        y_mod = model.forward_ids(cand, clk, proj_mode=mode)
        y_plan = plan.run(cand, clk).clone()
        same = bool(torch.equal(y_fwd, y_mod)) and (args.unfused or bool(torch.equal(y_fwd, y_plan)))
        # the stage breakdown comes from a separate pass with per-stage events:
        # an event between two kernels costs a few us of queue time (the empty
        # stage between two back-to-back events measures ~4.7 us), so the timed
        # steps run the product path without them
        n_ev = min(steps, 50)
        events = (fwd.make_events(n_ev) if not args.unfused else
                  [[torch.cuda.Event(enable_timing=True) for _ in range(n_st + 1)] for _ in range(n_ev)])
        # One batch repeated (not --stream): the step is captured once into a
        # HIP graph (the C ABI is capturable: no allocation, no sync) and
        # replayed, as a serving loop would; the eager loop is timed beside it.
        graph = None
        graphs, gstreams = [], []
        if not args.unfused and not args.stream and len(full) == 1 and not args.no_graph:
            # (--inflight K: K forwards, each with its own workspace, logits,
            # graph and stream; replayed in turn)
            fwds = [fwd] + [TimedForward(model, B, C, N_CLICKED, L, proj_mode=mode)
                            for _ in range(max(1, args.inflight) - 1)]
            for f in fwds:
                g = capture_graph(f, cand, clk, device)
                f.logits.fill_(float("nan"))     # the replay must recompute them
                g.replay()
                torch.cuda.synchronize()
                same = same and bool(torch.equal(f.logits, y_fwd))
                graphs.append(g)
                gstreams.append(torch.cuda.Stream(device))
            graph = graphs[0]
        eager_ms = None
        if graph is not None:
            torch.cuda.synchronize()
            te = time.perf_counter()
            run_steps(fwd, full, steps)
            torch.cuda.synchronize()
            eager_ms = (time.perf_counter() - te) / steps * 1e3
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None and len(graphs) > 1:
            cur = torch.cuda.current_stream(device)
            for st in gstreams:
                st.wait_stream(cur)
            for k in range(steps):
                with torch.cuda.stream(gstreams[k % len(graphs)]):
                    graphs[k % len(graphs)].replay()
        elif graph is not None:
            for _ in range(steps):
                graph.replay()
        else:
            run_steps(fwd, full, steps)
        if args.stream and tail_fwd is not None and steps == len(full):
            tail_fwd.run(*tail[0])
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    if dist:
        from newsrecommendationsystem_amd.distributed import max_over_ranks
        elapsed = max_over_ranks(elapsed, device)

    if args.dump_logits:
        # untimed: every batch of this rank's shard once, logits by impression
        # index -- from the timed path itself (the captured graph's replay when
        # the step is a graph replay: its logits buffer is poisoned first)
        import numpy as np
        with torch.no_grad():
            if graph is not None:
                fwd.logits.fill_(float("nan"))
                graph.replay()
                torch.cuda.synchronize()
                ys = [fwd.logits.clone()]
            else:
                ys = [fwd.run(*b).clone() for b in full] + ([tail_fwd.run(*tail[0]).clone()] if tail_fwd else [])
        n_done = sum(y.shape[0] for y in ys)
        np.savez(f"{args.dump_logits}.rank{rank}.npz", idx=idx[:n_done].cpu().numpy(),
                 logits=torch.cat(ys).float().cpu().numpy())
    # config 5's collective (the FedAvg parameter all-reduce over the group),
    # after the timed region: a multi-rank run measures its xGMI cost too
    fedavg = fedavg_sync_leg(model, device, dist) if dist else None
    with torch.no_grad():
        run_steps(fwd, full, n_ev, events)
        torch.cuda.synchronize()
    stage_ms = {st: 0.0 for st in stages}
    for ev in events:
        for i, st in enumerate(stages):
            stage_ms[st] += ev[i].elapsed_time(ev[i + 1])
    stage_ms = {st: v / n_ev for st, v in stage_ms.items()}
    # titles the news tail encodes per step (nrms_forward orders titles
    # [clicked | candidates]): with padding-title dedupe (library default,
    # nrms_set_title_dedupe) the all-zero titles count once (rep = the first);
    # with token compaction (nrms_set_token_compaction) a title is encoded on
    # Le = c + (c < 20) distinct q|k|v rows, c = its real (non-zero) tokens
    lib = Nat.load()
    compact = bool(lib.nrms_set_token_compaction(1))
    lib.nrms_set_token_compaction(int(compact))
    all_titles = torch.cat([clk.reshape(-1, L), cand.reshape(-1, L)])
    n_titles = all_titles.shape[0]
    cnt = (all_titles != 0).sum(-1)
    pad = cnt == 0
    n_pad = int(pad.sum())
    le = torch.where(cnt < L, cnt + 1, cnt) if compact else torch.full_like(cnt, L)
    le_enc = torch.cat([le[~pad], le[pad][:1]])   # the rep: one all-padding title
    n_enc = int(le_enc.numel())
    news_rows = (int(le_enc.sum()), int((le_enc * le_enc).sum()))
    # clicked rows the UserEncoder projects: the copied padding rows are skipped
    n_clk = clk.shape[0] * N_CLICKED
    clk_pad = int(pad[:n_clk].sum())
    n_user = n_clk - max(clk_pad - 1, 0) if not args.unfused else n_clk
    # UserEncoder rows: with compaction a user is encoded on Le = real + (1 if
    # any padding) rows (fused_user_kernel, UF_COMPACT), else on N
    real = (~pad[:n_clk]).view(-1, N_CLICKED).sum(-1)
    ule = torch.where(real < N_CLICKED, real + 1, real) if compact else torch.full_like(real, N_CLICKED)
    user_rows = (int(ule.sum()), int((ule * ule).sum()))
    work = (plan.work(titles_encoded=n_enc, user_rows_projected=n_user, news_rows=news_rows,
                      user_rows=user_rows) if not args.unfused else plan.work())
    dom = max(stage_ms, key=stage_ms.get)
    w = work[dom]
    t_dom = stage_ms[dom] / 1e3
    floor = issue_floor_ms(dom, w, args.gemm)
    bytes_floor = bytes_floor_ms(w)
    # the binding floor: the larger of the instruction-issue floor (the
    # matrix instructions the kernel actually issues, at their dense peaks)
    # and the bytes floor (algorithmic bytes at 8 TB/s)
    if floor is not None and floor > bytes_floor:
        # peak = the kernel's algorithmic FLOP over its issue floor: the rate of
        # its own instruction mix (split GEMM products at 2.5 PF, f32 at 157.3 TF)
        achieved, peak, unit, bound = (w["flop"] / t_dom / 1e12, w["flop"] / (floor * 1e-3) / 1e12,
                                       "TFLOP/s", "mfma")
    else:
        achieved, peak, unit, bound = w["bytes"] / t_dom / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"

    ms_per_step = elapsed / steps * 1e3
    if args.stream:
        done = (steps * B + (tail[0][0].shape[0] if tail and steps == len(full) else 0))
        if dist:
            from newsrecommendationsystem_amd.distributed import sum_over_ranks
            done = sum_over_ranks(done, device)
        value = done / elapsed
    else:
        value = world * B * steps / elapsed
    # every stage's floors (instruction issue, algorithmic bytes at 8 TB/s),
    # the binding one and the fraction of it achieved; their sum is the step's
    stage_floor = {}
    step_floor = 0.0
    for st_name, ms in stage_ms.items():
        if st_name in work:
            fl = issue_floor_ms(st_name, work[st_name], args.gemm)
            bf = bytes_floor_ms(work[st_name])
            bind = max(fl or 0.0, bf)
            if ms > 0.002:   # (an empty event pair: stage folded into another launch)
                step_floor += bind
            stage_floor[st_name] = {"issue_floor_ms": None if fl is None else round(fl, 4),
                                    "bytes_floor_ms": round(bf, 4),
                                    "bound": "mfma" if (fl or 0.0) > bf else "hbm",
                                    "floor_ms": round(bind, 4), "frac": round(bind / ms, 4) if ms > 0 else None}
    sq = load_sq(dom)
    traffic = load_traffic(dom)
    roofline = {"kernel": dom, "bound": bound, "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": unit,
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "algorithmic_per_launch": {"flop": w["flop"], "bytes": w["bytes"]},
                "bytes_floor_ms": round(bytes_floor, 4),
                "peak_note": ("bound = the larger of the kernel's instruction-issue floor and its bytes floor "
                              "(algorithmic bytes at 8 TB/s); frac = that floor / the measured launch time. "
                              "hbm: achieved = algorithmic bytes / launch time. mfma: achieved = algorithmic "
                              "fp32 FLOP / launch time, peak = those FLOP / the issue floor (the rate of the "
                              "kernel's own instruction mix)"),
                "fp32_flop_rate_vs_fp32_peak": round(w["flop"] / t_dom / 1e12 / PEAK_TFLOPS_F32, 4)}
    if traffic:
        roofline["traffic_vs_algorithmic"] = round(traffic / w["bytes"], 3)
    if floor is not None:
        # the fraction against the peak of the instructions the kernel actually
        # issues (its split GEMM's 16-bit products at 2.5 PF dense, the f32
        # attention / pooling at 157.3 TF)
        roofline["frac_vs_issued_peak"] = round(floor / stage_ms[dom], 4)
        roofline["issue_floor"] = {
            "ms": round(floor, 4), "frac": round(floor / stage_ms[dom], 4),
            "basis": (f"additive GEMM {args.gemm} ({ {'x6': 6, 'f16x3': 3}.get(args.gemm)} 16-bit products "
                      "per fp32 product) at 2.5 PF dense + attention contractions and pooling at 157.3 TF"
                      if args.gemm != "f32" else "all at 157.3 TF (f32 MFMA)"),
            "flop_split": w["split"]}
    if sq is not None:
        roofline["sq_counters"] = sq
    workload = ("BASELINE cfg4: full NRMS forward over the whole user-sharded stream "
                f"({idx.numel() if not dist else 'per-rank shards of'} impressions"
                f"{'' if dist else ' on this GPU'}), every title's vector produced (all-padding "
                "history titles encoded once per batch, see titles)"
                if args.stream else
                "BASELINE cfg3: full NRMS forward scoring (news+user encoder+click predictor), "
                "every title's vector produced (all-padding history titles encoded once per batch, see "
                "titles); batch = first B impressions of this rank's cfg4 user shard")
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "impressions/s", "n_gpus": world,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "strong" if args.stream else "weak", "vs_baseline": None,
        "dtype": {"f32": "fp32",
                  "x6": "fp32 (GEMMs: exact 3-way bf16 split, 6 products, fp32 accumulate)",
                  "f16x3": "fp32 (additive GEMM: 2-plane fp16 split, 22-bit operands, 3 products, fp32 "
                           "accumulate, out-of-fp16-range groups recomputed x6; Q|K|V projections: "
                           "power-of-two-scaled fp16 split, A in 3 pieces, W 22-bit, 3 products (4 where a W column "
                           "fits in 11 bits), fp32 "
                           "accumulate; UserEncoder additive GEMM: power-of-two-scaled 2-plane fp16 split, 3 products)"}[args.gemm],
        "data": "synthetic (MIND-shaped stream: counter-hash ids, random-init weights, N(0,1) embedding table)",
        "config": {"workload": workload, "global_batch": B * world,
                   "impressions_per_gpu": B, "candidates": C, "clicked": N_CLICKED,
                   "title_len": L, "vocab": V_WORDS, "d_model": D, "heads": 15,
                   "query_dim": 200, "proj_mode": args.proj, "gemm_arith": args.gemm,
                   "news_tail": "unfused" if args.unfused else "fused",
                   "stream": {"impressions": args.stream_impressions or S.N_IMPRESSIONS,
                              "users": S.N_USERS, "sharding": "user_id % world"},
                   "parallelism": f"user-shard x{world}",
                   "batches_in_flight": max(1, len(graphs))},
        "roofline": roofline,
        "titles": {"per_step": n_titles, "all_padding": n_pad, "encoded": n_enc,
                   "rows_encoded": news_rows[0], "rows_if_uncompacted": n_enc * L,
                   "token_compaction": compact,
                   "dedupe": "one all-padding title encoded per step, its vector read by the other "
                             "all-padding slots (bitwise identical logits: no_title_dedupe below)",
                   "compaction": "a title's id-0 tokens share one q|k|v row, encoded once with its "
                                 "multiplicity (news_fused.hip; fp32-rounding-level difference: "
                                 "no_token_compaction below)"},
        "stages_ms": {st: round(v, 4) for st, v in stage_ms.items()},
        "stages_issue_floor": stage_floor,
        "stages_issue_floor_note": ("issue_floor = the stage's algorithmic FLOP at the instruction rates it "
                                    "issues (split GEMMs: their 16-bit products at 2.5 PF dense; attention / "
                                    "pooling / exact f32 at 157.3 TF); bytes_floor = its algorithmic bytes at "
                                    "8 TB/s; floor = the larger (bound); frac = floor / measured stage time"),
        "step_floor": {"ms": round(step_floor, 4), "frac_of_ms_per_step": round(step_floor / ms_per_step, 4),
                       "note": "sum of the stages' binding floors against the timed step"},
        "user_rows_encoded": user_rows[0],
        "stages_note": f"HIP events recorded by the library between its stages, a separate pass of "
                       f"{n_ev} steps after the timed ones (events cost queue time, so the timed steps "
                       f"run without them). nrms_forward folds the click scores into the UserEncoder "
                       f"launch and the title classification into the pack launch and the vocabulary "
                       f"projection (qkv_news): 'score' is then an empty event pair, 'user_fused' "
                       f"includes the scoring",
        "user_rows_projected": n_user,
        "timed_path": (("nrms_forward (one C-ABI call) captured once in a HIP graph, replayed per step"
                        + (f"; {len(graphs)} batches in flight (--inflight: {len(graphs)} captured forwards, "
                           "each with its own workspace, logits and stream, replayed in turn; every step "
                           "still runs the whole forward of one batch)" if len(graphs) > 1 else ""))
                       if graph is not None else
                       "nrms_forward_timed without events (one C-ABI call per step)") if not args.unfused
                      else "ForwardPlan stage kernels (--unfused)",
        "eager": None if eager_ms is None else {
            "ms_per_step": round(eager_ms, 4), "impressions_per_s": round(B / (eager_ms / 1e3), 1),
            "note": "the same call issued from Python every step (no graph)"},
        "forward_paths_bitwise_equal": same,
        "graph_replay": graph is not None,
        "process_group": None if not dist else dist.get_backend(),
        "world_size": dist.get_world_size() if dist else 1,
        "launcher": os.environ.get("NRMS_BENCH_LAUNCHER",
                                   "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "none"),
    }
    if fedavg is not None:
        out["fedavg_sync"] = fedavg
    if args.as_shard:
        out["config"]["as_shard"] = args.as_shard
    if rank == 0 and world == 1 and not args.no_extras and not args.stream:
        out["gather_roofline"] = gather_hbm(device)
        out["news_encoder_cfg2"] = news_encoder_cfg2(model, device)
        if args.proj == "folded" and not args.unfused:
            dfwd = TimedForward(model, B, C, N_CLICKED, L, proj_mode=Nat.NRMS_PROJ_DIRECT)
            with torch.no_grad():
                y_d = dfwd.run(cand, clk).clone()
                dms = _time_launches(lambda: dfwd.run(cand, clk), 10, device)
            def variant(dedupe, compaction):
                pd, pc = lib.nrms_set_title_dedupe(dedupe), lib.nrms_set_token_compaction(compaction)
                try:
                    with torch.no_grad():
                        y = fwd.run(cand, clk).clone()
                        ms = _time_launches(lambda: fwd.run(cand, clk), 10, device)
                finally:
                    lib.nrms_set_title_dedupe(pd)
                    lib.nrms_set_token_compaction(pc)
                return y, ms
            y_c, cms = variant(1, 0)
            y_n, nms = variant(0, 0)
            out["no_token_compaction"] = {
                "ms_per_step": round(cms, 4), "impressions_per_s": round(B / (cms / 1e3), 1),
                "max_rel_diff_vs_default": float(((y_c - y_fwd).norm(dim=1) / y_fwd.norm(dim=1)).max()),
                "note": "every token of a title on its own q|k|v row (nrms_set_token_compaction(0))"}
            out["no_title_dedupe"] = {
                "ms_per_step": round(nms, 4), "impressions_per_s": round(B / (nms / 1e3), 1),
                "logits_bitwise_equal_to_no_token_compaction": bool(torch.equal(y_n, y_c)),
                "note": "every title and every token encoded, every clicked row projected separately "
                        "(nrms_set_title_dedupe(0) + nrms_set_token_compaction(0))"}
            out["direct_projection"] = {
                "ms_per_step": round(dms, 4), "impressions_per_s": round(B / (dms / 1e3), 1),
                "max_rel_diff_vs_folded": float(((y_d - y_fwd).norm(dim=1) / y_fwd.norm(dim=1)).max()),
                "note": "per-token Q|K|V projection (no vocabulary folding): the work SURVEY §8d's "
                        "789.6 MFLOP/impression unit describes"}
            del dfwd
    legs = {}
    if rank == 0 and world == 1 and not args.no_extras and not args.stream and not args.unfused:
        # the same step in the other GEMM arithmetics: x6 (exact bf16 products,
        # every operand split losslessly) beside the default's 22-bit operands
        legs = gemm_legs(model, cand, clk, mode, device, args.gemm, y_fwd)
        out["gemm_legs"] = legs
    if rank == 0 and world == 1 and not args.no_extras and not args.stream and not args.no_quality:
        # config 5's quality half (planted teacher, reference dimensions): FedAvg
        # on the HIP training path vs the reference op sequence + torch Adam,
        # both through evaluate()
        from newsrecommendationsystem_amd import quality
        out["fedavg_quality"] = quality.run_scaled()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.stream:
        cb, parity, ref_cpu = cpu_baseline(model, cand, clk)
        out["cpu_baseline"] = cb
        out["parity_vs_cpu"] = parity
        for g, leg in legs.items():
            yl = leg.pop("_logits").cpu()
            leg["max_normwise_rel_err_vs_cpu"] = float(
                ((yl - ref_cpu).norm(dim=1) / ref_cpu.norm(dim=1).clamp_min(1e-30)).max())
        out["auc_vs_cpu"] = eval_auc_check(model, device)
    if rank == 0 and world == 1 and not args.no_extras and not args.stream:
        out["eval_throughput"] = eval_throughput(model, device)
    out.setdefault("cpu_baseline", None)
    for leg in legs.values():
        leg.pop("_logits", None)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
