"""MIND-large-shaped synthetic impression stream (BASELINE config 4, SURVEY
§8d): 2,000,000 impressions over 1,000,000 user ids, sharded by
``user_id % world`` so every impression of a user, and the user's history,
lives on one rank (distributed.user_rank).

Everything is a counter-based hash (splitmix64 on int64 tensors), so any rank
generates any slice of the stream on its own device without materialising the
whole stream, and every rank sees the same stream:

  user(k)               = mix(stream 1, k) % n_users            impression k's user
  history length(u)     = 1 + mix(stream 2, u) % 50            U{1..50}, left-padded
  history title j of u  = title(stream 3, u * 64 + j)          j >= 50 - length
  candidate c of k      = title(stream 4, k * 8 + c)           c < 1 + K = 5
  title(s, key)         : length U{5..20}, ids U[1, V), right-padded with 0

Input layout per batch is the reference's forward contract
(src/dataset.py:64-85, src/model/NRMS/__init__.py:19-48): candidates
[B, 1+K, 20] (positive first) and clicked [B, 50, 20], int64.
"""
import torch

N_IMPRESSIONS = 2_000_000
N_USERS = 1_000_000
C, N_CLICKED, L = 5, 50, 20

_GOLDEN = -7046029254386353131     # 0x9E3779B97F4A7C15 as int64
_C1 = -4658895280553007687         # 0xBF58476D1CE4E5B9
_C2 = -7723592293110705685         # 0x94D049BB133111EB
_M = {30: (1 << 34) - 1, 27: (1 << 37) - 1, 31: (1 << 33) - 1, 11: (1 << 53) - 1}


def _srl(x, n):
    """Logical right shift of an int64 tensor (torch's >> is arithmetic)."""
    return (x >> n) & _M[n]


def mix(x):
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic)."""
    z = x + _GOLDEN
    z = (z ^ _srl(z, 30)) * _C1
    z = (z ^ _srl(z, 27)) * _C2
    return z ^ _srl(z, 31)


def _uniform_int(h, lo, hi):
    return lo + _srl(h, 11) % (hi - lo)


def _wrap64(v):
    """A Python int reduced to a signed int64 (two's-complement wrap), as the
    tensor arithmetic would wrap it."""
    return ((int(v) + (1 << 63)) % (1 << 64)) - (1 << 63)


def _key(seed, stream, x):
    # the seed term wraps to int64 first: any seed is valid (unchanged values
    # for the small seeds, where nothing wrapped)
    return mix(mix(x + _wrap64((seed * 1_000_003 + stream) * 0x1000000000)))


def impression_users(seed, k, n_users=N_USERS):
    """User id of each impression index in k (int64 tensor)."""
    return _uniform_int(_key(seed, 1, k), 0, n_users)


def titles(seed, stream, keys, V):
    """Token ids [.., L] of the titles with the given int64 keys."""
    h = _key(seed, stream, keys)
    length = _uniform_int(mix(h), 5, L + 1)
    pos = torch.arange(L, device=keys.device, dtype=torch.int64)
    tok = _uniform_int(mix(h.unsqueeze(-1) + pos + 1), 1, V)
    return torch.where(pos < length.unsqueeze(-1), tok, torch.zeros_like(tok))


def batch(seed, k, V, n_users=N_USERS):
    """The impressions with indices k (int64 [B]) -> (candidates [B, C, L],
    clicked [B, 50, L]) on k's device."""
    u = impression_users(seed, k, n_users)
    hist = _uniform_int(_key(seed, 2, u), 1, N_CLICKED + 1)
    j = torch.arange(N_CLICKED, device=k.device, dtype=torch.int64)
    clk = titles(seed, 3, u.unsqueeze(-1) * 64 + j, V)
    pad = j.unsqueeze(0) < (N_CLICKED - hist).unsqueeze(-1)
    clk = torch.where(pad.unsqueeze(-1), torch.zeros_like(clk), clk)
    c = torch.arange(C, device=k.device, dtype=torch.int64)
    cand = titles(seed, 4, k.unsqueeze(-1) * 8 + c, V)
    return cand.contiguous(), clk.contiguous()


def shard(seed, rank, world, n_impressions=N_IMPRESSIONS, n_users=N_USERS, device="cpu"):
    """Indices (int64, ascending) of the stream's impressions whose user this
    rank owns: user_id % world == rank."""
    k = torch.arange(n_impressions, device=device, dtype=torch.int64)
    if world <= 1:
        return k
    return k[impression_users(seed, k, n_users) % world == rank]
