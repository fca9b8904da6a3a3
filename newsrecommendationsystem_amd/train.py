"""Training step of src/train.py and the federated-averaging loop of
BASELINE config 5 (one process per GPU, local Adam steps, parameter
all-reduce over RCCL every E steps).

On a GPU the training step runs the HIP training kernels (train_hip.py:
train-mode forward with dropout, backward, Adam). The functions below are the
reference's own op sequence on ATen autograd: the CPU path, and the GPU
tests' reference for the HIP gradients (tests/test_gpu_train.py). Config 5's
FedAvg exchange: `FedAvg.sync()` averages the 21,955,400 fp32 parameters
(87.8 MB) with one all-reduce. The reference has no federated averaging at all
(SURVEY §0 finding 2), so there is no oracle for the averaged trajectory; the
tests check the exchange itself (every rank ends with the exact mean) and the
single-process step against the CPU restatement's autograd.

Semantics kept from the reference:
  * dropout p = config.dropout_probability on the embedding output and on the
    MHSA output (src/model/NRMS/news_encoder.py:38-45), identity in eval;
  * raw-exp attention normalisation (multihead_self.py:15-23);
  * CrossEntropyLoss against class 0 = the positive candidate first
    (src/train.py:126,205-206); Adam(lr = config.learning_rate) (:127);
  * nn.Embedding(padding_idx=0): row 0 receives no gradient.
"""
import math

import torch
import torch.nn.functional as F


def _mhsa(x, m):
    # src/model/general/attention/multihead_self.py:46-75 (+ :15-23)
    b = x.size(0)
    h, dk = m.num_attention_heads, m.d_k
    q = m.W_Q(x).view(b, -1, h, dk).transpose(1, 2)
    k = m.W_K(x).view(b, -1, h, dk).transpose(1, 2)
    v = m.W_V(x).view(b, -1, h, dk).transpose(1, 2)
    e = torch.exp(torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(dk))
    a = e / (e.sum(dim=-1, keepdim=True) + 1e-8)
    return torch.matmul(a, v).transpose(1, 2).contiguous().view(b, -1, h * dk)


def _additive(x, m):
    # src/model/general/attention/additive.py:27-53
    t = torch.tanh(m.linear(x))
    w = F.softmax(torch.matmul(t, m.attention_query_vector), dim=1)
    return torch.bmm(w.unsqueeze(1), x).squeeze(1)


def news_encode_autograd(ne, ids, training=True):
    """NewsEncoder.forward (news_encoder.py:27-48) with autograd."""
    p = ne.config.dropout_probability
    x = F.dropout(ne.word_embedding(ids), p=p, training=training)
    h = F.dropout(_mhsa(x, ne.multihead_self_attention), p=p, training=training)
    return _additive(h, ne.additive_attention)


def user_encode_autograd(ue, clicked_vec):
    """UserEncoder.forward (user_encoder.py:15-26) with autograd."""
    return _additive(_mhsa(clicked_vec, ue.multihead_self_attention), ue.additive_attention)


def forward_autograd(model, cand_ids, clicked_ids, training=True):
    """NRMS.forward (src/model/NRMS/__init__.py:19-48) with autograd: all
    B*(C+N) titles go through the encoder in one call (the reference encodes the
    55 slots one by one; per-title results and the dropout distribution are the
    same)."""
    ne, ue = model.news_encoder, model.user_encoder
    dev = ne.word_embedding.weight.device
    cand = cand_ids.to(dev)
    clk = clicked_ids.to(dev)
    B, C, L = cand.shape
    n_clicked = clk.shape[1]
    vec = news_encode_autograd(ne, torch.cat([cand.reshape(B * C, L), clk.reshape(B * n_clicked, L)]),
                               training)
    D = vec.shape[-1]
    cand_vec = vec[:B * C].view(B, C, D)
    clk_vec = vec[B * C:].view(B, n_clicked, D)
    user = user_encode_autograd(ue, clk_vec)
    return torch.bmm(cand_vec, user.unsqueeze(-1)).squeeze(-1)


def loss_fn(logits):
    """CrossEntropyLoss vs class 0 (src/train.py:205-206)."""
    return F.cross_entropy(logits, torch.zeros(logits.shape[0], dtype=torch.long,
                                               device=logits.device))


def train_step(model, optimizer, cand_ids, clicked_ids):
    """One iteration of the loop body of src/train.py:202-236. On a GPU the
    forward/backward are the HIP training kernels (model.forward_ids in train
    mode -> train_hip.NRMSTrain); on the CPU, ATen autograd."""
    model.train()
    logits = model.forward_ids(cand_ids, clicked_ids)
    loss = loss_fn(logits)
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return loss.detach()


class FedAvg:
    """Federated averaging of the model parameters over a process group: every
    `every` local steps, one all-reduce of the flattened parameters (RCCL
    over xGMI when the group's backend is "nccl", gloo on CPU), divided by
    the world size. Adam moments stay local (each client keeps its own
    optimizer state, as in FedAvg with client-side adaptive optimisers)."""

    def __init__(self, model, every, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.every = int(every)
        self.params = [p for p in model.parameters()]
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, dtype=torch.float32, device=self.params[0].device)
        self.world = dist.get_world_size(group)
        self.steps = 0

    @torch.no_grad()
    def sync(self):
        off = 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            off += k
        from .distributed import all_reduce_
        all_reduce_(self.flat, self.group)
        self.flat.div_(self.world)
        off = 0
        for p in self.params:
            k = p.numel()
            p.copy_(self.flat[off:off + k].view_as(p))
            off += k

    def step(self):
        """Call after each local optimizer step; syncs every `every` steps."""
        self.steps += 1
        if self.every > 0 and self.steps % self.every == 0:
            self.sync()
            return True
        return False


def make_optimizer(model):
    """Adam(lr = config.learning_rate) (src/train.py:127): the HIP update
    (train_hip.HipAdam, same state keys) on a GPU, torch.optim.Adam on CPU."""
    if next(model.parameters()).is_cuda:
        from .train_hip import HipAdam
        return HipAdam(model.parameters(), lr=model.config.learning_rate)
    return torch.optim.Adam(model.parameters(), lr=model.config.learning_rate)


def synthetic_train_batches(seed, n_batches, B, V, C=3, N=50, L=20, device="cpu"):
    """MIND-shaped training batches (src/dataset.py:64-85 contract): 1 positive
    + K negatives per row (positive first), history left-padded with zero
    titles."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        ids = torch.randint(1, V, (B, C + N, L), generator=g)
        lens = torch.randint(5, L + 1, (B, C + N, 1), generator=g)
        ids = torch.where(torch.arange(L)[None, None] < lens, ids, torch.zeros_like(ids))
        hist = torch.randint(1, N + 1, (B, 1), generator=g)
        pad = torch.arange(N)[None] < (N - hist)
        clk = torch.where(pad[:, :, None], torch.zeros_like(ids[:, C:]), ids[:, C:])
        out.append((ids[:, :C].contiguous().to(device), clk.contiguous().to(device)))
    return out


def _main():
    """python -m newsrecommendationsystem_amd.train [--steps 20] [--batch 128] [--every 5]
    Under torch.distributed.run: FedAvg across ranks (config 5 shape); prints
    one JSON line on rank 0 with steps/s, sync time and the final loss."""
    import argparse
    import json
    import time

    from .config import NRMSConfig
    from .distributed import init_from_env
    from .nrms import NRMS

    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--aten", action="store_true", help="ATen autograd + torch Adam instead of HIP")
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    rank, world, local, distributed = init_from_env()
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    torch.manual_seed(0)                        # identical initial weights on every rank

    class Cfg(NRMSConfig):
        hip_train = not a.aten
    model = NRMS(Cfg, torch.randn(NRMSConfig.num_words, 300)).to(dev)
    opt = (torch.optim.Adam(model.parameters(), lr=Cfg.learning_rate) if a.aten
           else make_optimizer(model))
    fed = FedAvg(model, a.every) if distributed else None
    batches = synthetic_train_batches(100 + rank, a.steps + a.warmup, a.batch, NRMSConfig.num_words,
                                      device=dev)
    for cand, clk in batches[:a.warmup]:
        train_step(model, opt, cand, clk)
    batches = batches[a.warmup:]
    sync_t = 0.0
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for cand, clk in batches:
        loss = train_step(model, opt, cand, clk)
        if fed is not None:
            if dev.type == "cuda":
                torch.cuda.synchronize()
            ts = time.perf_counter()
            if fed.step() and dev.type == "cuda":
                torch.cuda.synchronize()
            sync_t += time.perf_counter() - ts
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"mode": ("train (HIP kernels)" if dev.type == "cuda" and not a.aten
                                   else "train (ATen autograd)") + " + FedAvg", "world": world, "steps": a.steps,
                          "batch_per_rank": a.batch, "fedavg_every": a.every,
                          "steps_per_s": a.steps / dt, "samples_per_s": world * a.batch * a.steps / dt,
                          "fedavg_sync_s_total": sync_t, "final_loss": float(loss),
                          "param_bytes": int(sum(p.numel() for p in model.parameters()) * 4)}))


if __name__ == "__main__":
    _main()
