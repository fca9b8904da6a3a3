"""Deterministic parameter / input generator for the NRMS oracle (test infra).

numpy's Generator streams are not guaranteed stable across numpy releases, so
fixtures are regenerated from this splitmix64 counter generator instead: the
same (seed, stream, shape) always yields the same float32 values on every
machine. Fixtures then only need to hold ids and expected outputs.

Distributions follow the reference's initialisers:
  * word embedding  ~ N(0,1), row 0 NOT zeroed
        (src/data_preprocess.py:272-277, src/model/NRMS/news_encoder.py:14-20)
  * W_Q/W_K/W_V     xavier_uniform(gain=1): U(-sqrt(6/600), +sqrt(6/600))
        (src/model/general/attention/multihead_self.py:41-44)
  * Linear biases   U(-1/sqrt(fan_in), +1/sqrt(fan_in))  (torch nn.Linear default)
  * additive linear U(-1/sqrt(300), +1/sqrt(300))         (nn.Linear default)
  * query vector    U(-0.1, 0.1)  (src/model/general/attention/additive.py:19-20)
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def uniform01(seed, stream, n):
    """n float64 values in [0,1) from counter (seed, stream, i)."""
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(seed) * np.uint64(0x100000001B3) ^ np.uint64(stream))
        ctr = np.arange(n, dtype=np.uint64) + base
        bits = _splitmix64(ctr) >> np.uint64(11)
    return bits.astype(np.float64) * (1.0 / (1 << 53))


def uniform(seed, stream, shape, lo, hi):
    n = int(np.prod(shape))
    return (lo + (hi - lo) * uniform01(seed, stream, n)).astype(np.float32).reshape(shape)


def normal(seed, stream, shape, scale=1.0):
    n = int(np.prod(shape))
    m = (n + 1) // 2
    u1 = uniform01(seed, stream, m)
    u2 = uniform01(seed, stream + 0x5151, m)
    r = np.sqrt(-2.0 * np.log1p(-u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])[:n]
    return (scale * z).astype(np.float32).reshape(shape)


def randint(seed, stream, shape, lo, hi):
    """Integers uniform in [lo, hi)."""
    n = int(np.prod(shape))
    u = uniform01(seed, stream, n)
    return (lo + np.floor(u * (hi - lo))).astype(np.int64).reshape(shape)


def encoder_params(seed, base_stream, D=300, Q=200):
    """MHSA + additive parameters for one encoder, keyed like the reference."""
    xb = float(np.sqrt(6.0 / (D + D)))
    lb = float(1.0 / np.sqrt(D))
    s = base_stream
    p = {}
    for i, name in enumerate(("W_Q", "W_K", "W_V")):
        p[f"multihead_self_attention.{name}.weight"] = uniform(seed, s + 2 * i, (D, D), -xb, xb)
        p[f"multihead_self_attention.{name}.bias"] = uniform(seed, s + 2 * i + 1, (D,), -lb, lb)
    p["additive_attention.attention_query_vector"] = uniform(seed, s + 10, (Q,), -0.1, 0.1)
    p["additive_attention.linear.weight"] = uniform(seed, s + 11, (Q, D), -lb, lb)
    p["additive_attention.linear.bias"] = uniform(seed, s + 12, (Q,), -lb, lb)
    return p


def nrms_state(seed, V, D=300, Q=200):
    """Full NRMS state_dict (numpy float32) with the reference's key names
    (src/model/NRMS/__init__.py:12-17)."""
    sd = {"news_encoder.word_embedding.weight": normal(seed, 1, (V, D))}
    for k, v in encoder_params(seed, 100, D, Q).items():
        sd["news_encoder." + k] = v
    for k, v in encoder_params(seed, 200, D, Q).items():
        sd["user_encoder." + k] = v
    return sd


def titles(seed, stream, n, V, L=20, min_len=5):
    """Synthetic titles per SURVEY §8d: length U{min_len..L}, ids U[1,V),
    right-padded with 0 (src/data_preprocess.py:115,132-139)."""
    ids = randint(seed, stream, (n, L), 1, V)
    lens = randint(seed, stream + 1, (n,), min_len, L + 1)
    mask = np.arange(L)[None, :] < lens[:, None]
    return np.where(mask, ids, 0).astype(np.int64)


def impressions(seed, stream, B, V, C=5, N=50, L=20):
    """Forward-semantics batch (src/dataset.py:64-85): C candidate titles and
    the first N clicked titles, history left-padded with all-zero titles.
    Returns (candidates [B,C,L], clicked [B,N,L], history_lengths [B])."""
    cand = titles(seed, stream, B * C, V, L).reshape(B, C, L)
    clk = titles(seed, stream + 2, B * N, V, L).reshape(B, N, L)
    hist = randint(seed, stream + 4, (B,), 1, N + 1)
    pad = np.arange(N)[None, :] < (N - hist)[:, None]
    clk = np.where(pad[:, :, None], 0, clk).astype(np.int64)
    return cand, clk, hist
