"""CPU restatement of the NRMS path as the reference's ATen op sequence —
TEST INFRASTRUCTURE and the timed CPU baseline (bench.py ``cpu_baseline``,
kind "port").

The reference itself cannot travel to the GPU box, so this functional
restatement dispatches the same ATen ops in the same order as
src/model/NRMS/* and src/model/general/* (F.embedding, F.linear, matmul,
exp, sum, div, softmax, bmm) on CPU tensors. tests/test_oracle_golden.py
checks it against the golden vectors captured from the reference.
"""
import numpy as np
import torch
import torch.nn.functional as F

N_HEADS = 15


def _mhsa(x, sd, prefix, n_heads=N_HEADS):
    # src/model/general/attention/multihead_self.py:46-75 (+ :15-23)
    b = x.size(0)
    d = x.size(-1)
    dk = d // n_heads

    def proj(name):
        y = F.linear(x, sd[f"{prefix}.{name}.weight"], sd[f"{prefix}.{name}.bias"])
        return y.view(b, -1, n_heads, dk).transpose(1, 2)

    q, k, v = proj("W_Q"), proj("W_K"), proj("W_V")
    scores = torch.exp(torch.matmul(q, k.transpose(-1, -2)) / np.sqrt(dk))
    attn = scores / (torch.sum(scores, dim=-1, keepdim=True) + 1e-8)
    ctx = torch.matmul(attn, v)
    return ctx.transpose(1, 2).contiguous().view(b, -1, n_heads * dk)


def _additive(x, sd, prefix):
    # src/model/general/attention/additive.py:27-53
    t = torch.tanh(F.linear(x, sd[f"{prefix}.linear.weight"], sd[f"{prefix}.linear.bias"]))
    w = F.softmax(torch.matmul(t, sd[f"{prefix}.attention_query_vector"]), dim=1)
    return torch.bmm(w.unsqueeze(dim=1), x).squeeze(dim=1)


def news_encode(ids, sd):
    # src/model/NRMS/news_encoder.py:27-48 (eval: dropout is the identity)
    x = F.embedding(ids, sd["news_encoder.word_embedding.weight"], padding_idx=0)
    return _additive(_mhsa(x, sd, "news_encoder.multihead_self_attention"), sd,
                     "news_encoder.additive_attention")


def user_encode(clicked_vec, sd):
    # src/model/NRMS/user_encoder.py:15-26
    return _additive(_mhsa(clicked_vec, sd, "user_encoder.multihead_self_attention"), sd,
                     "user_encoder.additive_attention")


def click_score(news_vec, user_vec):
    # src/model/general/click_predictor/dot_product.py:8-19
    return torch.bmm(news_vec, user_vec.unsqueeze(dim=-1)).squeeze(dim=-1)


def forward(candidates, clicked, sd):
    """NRMS.forward (src/model/NRMS/__init__.py:19-48) over [B,C,L] / [B,N,L]
    id tensors, one encoder call per slot as the reference does."""
    cand = torch.stack([news_encode(candidates[:, i], sd) for i in range(candidates.size(1))], dim=1)
    clk = torch.stack([news_encode(clicked[:, i], sd) for i in range(clicked.size(1))], dim=1)
    return click_score(cand, user_encode(clk, sd))


def state_to_torch(sd):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}
