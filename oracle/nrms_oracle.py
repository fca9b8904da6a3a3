"""numpy restatement of the reference NRMS scoring path — TEST INFRASTRUCTURE.

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline as
the checker. Each function cites the reference lines it restates (paths
relative to the reference repo root). Eval-mode semantics throughout: the two
F.dropout calls of the NewsEncoder are the identity when ``training=False``
(src/model/NRMS/news_encoder.py:38-40,43-45).

``dt`` selects the arithmetic type (np.float32 to mirror the reference, or
np.float64 for a high-precision yardstick).
"""
import numpy as np

D_MODEL = 300
N_HEADS = 15
QUERY_DIM = 200


def embedding_gather(table, ids):
    """nn.Embedding forward (src/model/NRMS/news_encoder.py:38): a plain row
    gather. padding_idx=0 only affects gradients, so id 0 is gathered like any
    other id (row 0 is N(0,1) for pretrained tables: data_preprocess.py:272-277)."""
    ids = np.asarray(ids)
    if ids.size and (ids.min() < 0 or ids.max() >= table.shape[0]):
        raise IndexError("index out of range in self")
    return table[ids]


def linear(x, w, b, dt=np.float32):
    """nn.Linear: x @ w.T + b."""
    return x.astype(dt) @ w.astype(dt).T + b.astype(dt)


def raw_exp_attention(q, k, v, d_k, dt=np.float32):
    """ScaledDotProductAttention.forward (src/model/general/attention/
    multihead_self.py:15-23) with attn_mask=None: scores = QK^T / sqrt(d_k);
    exp WITHOUT max-subtraction; attn = e / (sum(e) + 1e-8); context = attn @ V.
    Overflow (score > ~88.7) gives inf/inf = NaN, all-underflow gives 0."""
    with np.errstate(over="ignore", invalid="ignore", under="ignore"):
        s = np.matmul(q, np.swapaxes(k, -1, -2)) / dt(np.sqrt(d_k))
        e = np.exp(s.astype(dt))
        a = e / (e.sum(axis=-1, keepdims=True) + dt(1e-8))
        return np.matmul(a, v).astype(dt)


def multihead_self_attention(x, p, prefix, n_heads=N_HEADS, dt=np.float32):
    """MultiHeadSelfAttention.forward (multihead_self.py:46-75), K=V=Q=x:
    three Linear projections, split into heads of d_k = d_model / n_heads
    (:31-33), raw-exp attention per head, heads concatenated in head order with
    no output projection, residual or norm (:74-75)."""
    n, L, d = x.shape
    dk = d // n_heads
    proj = []
    for name in ("W_Q", "W_K", "W_V"):
        y = linear(x.reshape(n * L, d), p[f"{prefix}.{name}.weight"], p[f"{prefix}.{name}.bias"], dt)
        proj.append(y.reshape(n, L, n_heads, dk).transpose(0, 2, 1, 3))
    ctx = raw_exp_attention(proj[0], proj[1], proj[2], dk, dt)
    return ctx.transpose(0, 2, 1, 3).reshape(n, L, d)


def additive_attention(x, p, prefix, dt=np.float32):
    """AdditiveAttention.forward (src/model/general/attention/additive.py:27-53):
    w = softmax_L(tanh(x W^T + b) . q) (standard max-subtracted softmax,
    :37-39), out = sum_l w_l x_l (:51-52)."""
    n, L, d = x.shape
    t = np.tanh(linear(x.reshape(n * L, d), p[f"{prefix}.linear.weight"], p[f"{prefix}.linear.bias"], dt))
    s = (t @ p[f"{prefix}.attention_query_vector"].astype(dt)).reshape(n, L)
    s = s - s.max(axis=1, keepdims=True)
    e = np.exp(s)
    w = (e / e.sum(axis=1, keepdims=True)).astype(dt)
    return np.einsum("nl,nld->nd", w, x.astype(dt)).astype(dt)


def news_encode(ids, sd, dt=np.float32):
    """NewsEncoder.forward (src/model/NRMS/news_encoder.py:27-48), eval mode:
    int64 [n, L] title ids -> [n, 300] news vectors."""
    x = embedding_gather(sd["news_encoder.word_embedding.weight"], ids).astype(dt)
    h = multihead_self_attention(x, sd, "news_encoder.multihead_self_attention", dt=dt)
    return additive_attention(h, sd, "news_encoder.additive_attention", dt)


def user_encode(clicked_vec, sd, dt=np.float32):
    """UserEncoder.forward (src/model/NRMS/user_encoder.py:15-26): MHSA over the
    N clicked-news vectors, then additive pooling: [B, N, 300] -> [B, 300]."""
    h = multihead_self_attention(np.asarray(clicked_vec, dtype=dt), sd,
                                 "user_encoder.multihead_self_attention", dt=dt)
    return additive_attention(h, sd, "user_encoder.additive_attention", dt)


def click_score(news_vec, user_vec, dt=np.float32):
    """DotProductClickPredictor.forward (src/model/general/click_predictor/
    dot_product.py:8-19): bmm([B,C,X], [B,X,1]) -> [B,C] logits (no sigmoid)."""
    return np.einsum("bcd,bd->bc", news_vec.astype(dt), user_vec.astype(dt)).astype(dt)


def forward(candidates, clicked, sd, dt=np.float32):
    """NRMS.forward (src/model/NRMS/__init__.py:19-48): candidates [B,C,L] and
    clicked [B,N,L] title ids -> logits [B,C]. Every slot is encoded (the
    reference loops over slots; the result is the same per slot)."""
    B, C, L = candidates.shape
    N = clicked.shape[1]
    cand_vec = news_encode(candidates.reshape(B * C, L), sd, dt).reshape(B, C, -1)
    clk_vec = news_encode(clicked.reshape(B * N, L), sd, dt).reshape(B, N, -1)
    user = user_encode(clk_vec, sd, dt)
    return click_score(cand_vec, user, dt)


def get_prediction(news_vector, user_vector, dt=np.float32):
    """NRMS.get_prediction (src/model/NRMS/__init__.py:73-84): [C,X],[X] -> [C]."""
    return click_score(news_vector[None], user_vector[None], dt)[0]


def normwise_rel_err(a, b):
    """Per-row ||a-b||_2 / ||b||_2 (SURVEY §8d parity criterion)."""
    a = np.asarray(a, dtype=np.float64).reshape(len(a), -1) if np.ndim(a) > 1 else np.asarray(a, np.float64)[None]
    b = np.asarray(b, dtype=np.float64).reshape(a.shape)
    den = np.linalg.norm(b, axis=1)
    num = np.linalg.norm(a - b, axis=1)
    return num / np.maximum(den, 1e-30)
