"""Config 5's quality half on a planted teacher: FedAvg training on the HIP
path against the same training on the CPU (ATen) path, both evaluated with
evaluate() (src/train.py:161-236 followed by src/evaluate.py:171-272).

BASELINE config 5 asks for "AUC on MIND-small dev"; MIND is not available
here or on the GPU box, so SURVEY §8d's fallback is used: a fixed random NRMS
(the teacher) labels a synthetic MIND-shaped corpus. Training batches follow
the src/dataset.py:64-85 contract (positive first, histories left-padded with
all-zero titles); the positive of each row is the teacher's top-scored of its
1 + K candidates. The eval split (news_parsed.tsv + behaviors.tsv in the
reference formats) draws its click labels from the teacher's logits.

Both students start from one initialisation (dropout 0, so no RNG enters the
step) and run the same FedAvg schedule: `world` clients, each with its own
batches and its own Adam, parameters averaged every `every` local steps
(train.FedAvg's exchange: the sum over clients divided by the count). The HIP
student runs the HIP training kernels + HipAdam (train_hip.py) on the GPU, the
CPU student the reference op sequence on ATen autograd + torch.optim.Adam
(train.py). Here the clients run in one process one after the other (the
exchange is the same arithmetic); tests/test_gpu_multiprocess.py runs the HIP
clients as two processes over a real process group.
"""
import copy
import tempfile
import time

import numpy as np
import torch

from . import data as Dt
from . import train as TR
from .config import NRMSConfig
from .evaluate import EvalPlan, evaluate, score_plan
from .nrms import NRMS


def make_config(V, lr=2e-3, dropout=0.0):
    """NRMSConfig for the planted-teacher runs: vocabulary V, dropout (0: no
    RNG in the step), learning rate lr (the reference's 1e-4 moves a random
    student too little in a few hundred steps to say anything about AUC)."""
    return type("QualityCfg", (NRMSConfig,), dict(num_words=V, dropout_probability=dropout, learning_rate=lr))


def model_from_seed(cfg, seed):
    torch.manual_seed(seed)
    return NRMS(cfg, torch.randn(cfg.num_words, 300) * 0.5)


def teacher_logits_fn(teacher):
    """teacher(corpus, impressions) -> per-impression logits (eval pipeline)."""
    def fn(corpus, imps):
        plan = EvalPlan(corpus, imps)
        sc, _ = score_plan(teacher, plan)
        sc = sc.cpu().numpy()
        return [sc[a:b] for a, b in zip(plan.offsets[:-1], plan.offsets[1:])]
    return fn


def teacher_batches(teacher, titles, seed, n_batches, B, C=3, N=50):
    """Training batches from the corpus titles [n_news, 20]: per row a history of
    U{1..N} clicked news (left-padded with all-zero titles, src/dataset.py:79-83)
    and C candidates, reordered so the teacher's top-scored one is first
    (class 0, src/train.py:205-206). CPU int64 tensors."""
    rng = np.random.default_rng(seed)
    dev = next(teacher.parameters()).device
    n_news, L = titles.shape
    out = []
    for _ in range(n_batches):
        cand = titles[rng.integers(0, n_news, (B, C))]
        clk = titles[rng.integers(0, n_news, (B, N))].copy()
        hist = rng.integers(1, N + 1, B)
        clk[np.arange(N)[None, :] < (N - hist)[:, None]] = 0
        with torch.no_grad():
            y = teacher.forward_ids(torch.from_numpy(cand), torch.from_numpy(clk)).cpu().numpy()
        order = np.argsort(-y, axis=1, kind="stable")
        cand = np.take_along_axis(cand, order[:, :, None], axis=1)
        out.append((torch.from_numpy(np.ascontiguousarray(cand)), torch.from_numpy(clk)))
    return out


def train_clients(init, client_batches, every, device):
    """FedAvg over len(client_batches) clients, each its own copy of `init`
    (on `device`) and its own optimizer (train.make_optimizer: HipAdam on a
    GPU, torch Adam on the CPU); after every `every` local steps the
    parameters of all clients are replaced by their mean. Returns (model,
    seconds spent in the local steps, steps taken per client)."""
    models = [copy.deepcopy(init).to(device) for _ in client_batches]
    opts = [TR.make_optimizer(m) for m in models]
    steps = len(client_batches[0])
    t_steps = 0.0
    for k in range(steps):
        for m, opt, batches in zip(models, opts, client_batches):
            cand, clk = batches[k]
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            TR.train_step(m, opt, cand.to(device), clk.to(device))
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t_steps += time.perf_counter() - t0
        if every > 0 and (k + 1) % every == 0:
            with torch.no_grad():
                for ps in zip(*[list(m.parameters()) for m in models]):
                    acc = ps[0].detach().clone()
                    for p in ps[1:]:
                        acc += p.detach()
                    acc /= len(ps)
                    for p in ps:
                        p.copy_(acc)
    return models[0], t_steps, steps


def setup(directory, V=5000, n_news=3000, n_users=800, n_impressions=1500, seed=0, lr=2e-3):
    """Teacher, the eval split written under `directory`, the corpus titles and
    the student initialisation."""
    cfg = make_config(V, lr)
    teacher = model_from_seed(cfg, 1000 + seed).cuda().eval()
    corpus, imps = Dt.synthetic_split(directory, seed=seed, n_news=n_news, n_users=n_users,
                                      n_impressions=n_impressions, V=V, teacher=teacher_logits_fn(teacher))
    student = model_from_seed(cfg, 2000 + seed)
    return cfg, teacher, corpus, np.asarray(corpus.titles, dtype=np.int64), student


def auc_of(model_state, cfg, directory):
    """evaluate() (the HIP eval pipeline) of a state dict on the split."""
    m = NRMS(cfg)
    m.load_state_dict(model_state)
    m = m.cuda().eval()
    return evaluate(m, directory)


def run(steps=32, every=4, world=2, B=16, C=3, seed=0, cpu=True):
    """Both students trained and evaluated; returns a JSON-able dict."""
    with tempfile.TemporaryDirectory() as d:
        cfg, teacher, corpus, titles, student = setup(d, seed=seed)
        client_batches = [teacher_batches(teacher, titles, 100 + 17 * r + seed, steps, B, C) for r in range(world)]
        init_auc = auc_of(student.state_dict(), cfg, d)
        hip, t_hip, n = train_clients(student, client_batches, every, torch.device("cuda"))
        hip_sd = {k: v.detach().cpu() for k, v in hip.state_dict().items()}
        auc_hip = auc_of(hip_sd, cfg, d)
        out = {"workload": (f"planted teacher: {world} FedAvg clients x {steps} local steps (batch {B}, "
                            f"1+K={C}, 50 clicked, V={cfg.num_words}, lr {cfg.learning_rate}, dropout 0, "
                            f"average every {every}); eval split {len(corpus.ids)} news, "
                            "labels ~ Bernoulli(sigmoid(teacher logit))"),
               "auc_init": init_auc[0], "auc_hip": auc_hip[0],
               "hip_train_steps_per_s": round(world * n / t_hip, 2)}
        if cpu:
            cpu_m, t_cpu, _ = train_clients(student, client_batches, every, torch.device("cpu"))
            cpu_sd = {k: v.detach().cpu() for k, v in cpu_m.state_dict().items()}
            auc_cpu = auc_of(cpu_sd, cfg, d)
            # (W_K's bias has an analytically zero gradient -- the normalisation
            # divides a key bias out -- so Adam turns either path's rounding
            # noise into +-lr steps there; it is left out of the comparison)
            diff = max(float((hip_sd[k] - cpu_sd[k]).norm() / cpu_sd[k].norm().clamp_min(1e-30))
                       for k in cpu_sd if not k.endswith("W_K.bias"))
            out.update({"auc_cpu": auc_cpu[0], "abs_diff_auc": abs(auc_hip[0] - auc_cpu[0]),
                        "tolerance": 0.002, "cpu_train_steps_per_s": round(world * n / t_cpu, 2),
                        "max_normwise_param_diff_hip_vs_cpu_excl_WK_bias": diff,
                        "mrr_hip": auc_hip[1], "mrr_cpu": auc_cpu[1]})
        return out


# ---------------------------------------------------------------- config 5 at scale
def teacher_batches_device(teacher, titles, seed, n_batches, B, C=3, N=50):
    """teacher_batches on the device (titles: int64 [n_news, 20] there): per
    row U{1..N} clicked news left-padded with all-zero titles
    (src/dataset.py:79-83) and C candidates ordered by the teacher's score,
    positive first (src/train.py:205-206)."""
    dev = titles.device
    g = torch.Generator(device=dev).manual_seed(seed)
    n_news, L = titles.shape
    out = []
    for _ in range(n_batches):
        cand = titles[torch.randint(0, n_news, (B, C), generator=g, device=dev)]
        clk = titles[torch.randint(0, n_news, (B, N), generator=g, device=dev)]
        hist = torch.randint(1, N + 1, (B, 1), generator=g, device=dev)
        clk = torch.where((torch.arange(N, device=dev)[None] < (N - hist))[:, :, None], torch.zeros_like(clk), clk)
        with torch.no_grad():
            y = teacher.forward_ids(cand, clk)
        order = torch.argsort(-y, dim=1, stable=True)
        cand = torch.gather(cand, 1, order[:, :, None].expand(-1, -1, L))
        out.append((cand.contiguous(), clk.contiguous()))
    return out


def _fedavg_(models):
    """Replace every client's parameters by the clients' mean (train.FedAvg's
    exchange: sum over clients / count)."""
    with torch.no_grad():
        for ps in zip(*[list(m.parameters()) for m in models]):
            acc = ps[0].detach().clone()
            for p in ps[1:]:
                acc += p.detach()
            acc /= len(ps)
            for p in ps:
                p.copy_(acc)


def train_clients_reference(init, client_batches, every, device):
    """The same FedAvg schedule on the reference's op sequence (train.py:
    forward_autograd, ATen autograd, CrossEntropy vs class 0) with
    torch.optim.Adam, on `device`. With dropout p > 0 the step takes the HIP
    step's dropout sample: its masks come from the HIP generator with the same
    per-call seed the HIP student uses (1, 2, ... per client, NRMS.forward_ids)
    and enter as explicit multiplicative masks (train.forward_autograd_masked)."""
    models = [copy.deepcopy(init).to(device) for _ in client_batches]
    opts = [torch.optim.Adam(m.parameters(), lr=m.config.learning_rate) for m in models]
    p = float(init.config.dropout_probability)
    steps = len(client_batches[0])
    t_steps = 0.0
    for k in range(steps):
        for m, opt, batches in zip(models, opts, client_batches):
            cand, clk = (t.to(device) for t in batches[k])
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            m.train()
            if p > 0:
                B, C, L = cand.shape
                masks = TR.hip_dropout_masks(B * (C + clk.shape[1]) * L, 300, p, k + 1, device)
                logits = TR.forward_autograd_masked(m, cand, clk, masks)
            else:
                logits = TR.forward_autograd(m, cand, clk, training=False)
            loss = TR.loss_fn(logits)
            opt.zero_grad()
            loss.backward()
            opt.step()
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t_steps += time.perf_counter() - t0
        if every > 0 and (k + 1) % every == 0:
            _fedavg_(models)
    return models[0], t_steps, steps


def run_scaled(steps=320, every=10, world=2, B=128, C=3, V=70976, n_news=20000, dropouts=(0.0, 0.2),
               lr=2e-3, seed=0, temperature=0.5, eval_impressions=4000):
    """BASELINE config 5's quality half at the reference's dimensions: V =
    70,976 words, batch 128 (src/config.py:18), 1 + K = 3 candidates, 50
    clicked, `world` FedAvg clients x `steps` local steps, parameters averaged
    every `every` steps; the HIP student (HIP training kernels + HipAdam)
    against the reference student (the reference's op sequence on ATen
    autograd + torch.optim.Adam, on the GPU as src/train.py:24 selects when
    one is present), both from one initialisation on the same batches, both
    evaluated with evaluate() on a planted-teacher split. One run per dropout
    probability; with p > 0 the reference student takes the HIP masks."""
    dev = torch.device("cuda")
    res = {"workload": (f"planted teacher: {world} FedAvg clients x {steps} local steps, batch {B}, 1+K={C}, "
                        f"50 clicked, V={V}, {n_news} news, lr {lr}, FedAvg every {every} steps; eval split "
                        f"{eval_impressions} impressions, labels ~ Bernoulli(sigmoid(teacher logit / {temperature}))"),
           "reference_path": "src/train.py loop body on ATen autograd + torch.optim.Adam, on the GPU "
                             "(src/train.py:24 device selection)",
           "runs": []}
    with tempfile.TemporaryDirectory() as d:
        cfg0 = make_config(V, lr)
        teacher = model_from_seed(cfg0, 1000 + seed).to(dev).eval()
        corpus, imps = Dt.synthetic_split(d, seed=seed, n_news=n_news, n_users=3000,
                                          n_impressions=eval_impressions, V=V,
                                          teacher=teacher_logits_fn(teacher), temperature=temperature)
        titles = torch.from_numpy(np.asarray(corpus.titles, dtype=np.int64)).to(dev)
        client_batches = [teacher_batches_device(teacher, titles, 100 + 17 * r + seed, steps, B, C)
                          for r in range(world)]
        for p in dropouts:
            cfg = make_config(V, lr, dropout=p)
            torch.manual_seed(2000 + seed)
            student = NRMS(cfg, torch.randn(V, 300) * 0.5)
            init_auc = auc_of(student.state_dict(), cfg, d)
            hip, t_hip, n = train_clients(student, client_batches, every, dev)
            hip_sd = {k: v.detach().cpu() for k, v in hip.state_dict().items()}
            del hip
            ref, t_ref, _ = train_clients_reference(student, client_batches, every, dev)
            ref_sd = {k: v.detach().cpu() for k, v in ref.state_dict().items()}
            del ref
            a_hip, a_ref = auc_of(hip_sd, cfg, d), auc_of(ref_sd, cfg, d)
            diff = max(float((hip_sd[k] - ref_sd[k]).norm() / ref_sd[k].norm().clamp_min(1e-30))
                       for k in ref_sd if not k.endswith("W_K.bias"))
            res["runs"].append({
                "dropout": p, "auc_init": init_auc[0], "auc_hip": a_hip[0], "auc_reference": a_ref[0],
                "auc_lift_hip": a_hip[0] - init_auc[0], "abs_diff_auc": abs(a_hip[0] - a_ref[0]),
                "tolerance": 0.002, "mrr_hip": a_hip[1], "mrr_reference": a_ref[1],
                "max_normwise_param_diff_excl_WK_bias": diff,
                "hip_train_steps_per_s": round(world * n / t_hip, 1),
                "reference_train_steps_per_s": round(world * n / t_ref, 1)})
            torch.cuda.empty_cache()
    return res
