"""Multi-GPU layout of the scoring path: one process per GPU,
weights replicated, impressions sharded by user so a user's history lives on
one rank; no collective on the data path. The only collective is the final
reduction of the per-impression metric sums (5 fp64 words per rank), over
RCCL (backend "nccl" on ROCm) between GPUs or gloo on CPU.

The reference has no distributed code (SURVEY §0 finding 1); this module is
new, and tests/test_distributed_cpu.py covers it with world_size 2 on gloo.
"""
import os
import re
import zlib

import torch


_DIGITS = re.compile(r"^[A-Za-z_]*(\d+)$")


def user_rank(user, world):
    """Owner rank of a user: user_id % world for integer
    ids and for MIND-style ids such as "U13740" (the number after the prefix);
    any other string by a stable hash (Python's hash() is salted per process)."""
    if isinstance(user, int):
        return user % world
    m = _DIGITS.match(str(user))
    if m:
        return int(m.group(1)) % world
    return zlib.crc32(str(user).encode()) % world


def shard_impressions(impressions, rank, world):
    """The impressions whose user this rank owns, in their original order (a
    data.BehaviorsTable stays a table)."""
    from .data import BehaviorsTable
    if isinstance(impressions, BehaviorsTable):
        if world <= 1:
            return impressions
        import numpy as np
        mine = np.array([user_rank(u, world) == rank for u in impressions.users()], dtype=bool)
        return impressions.select(np.flatnonzero(mine))
    if world <= 1:
        return list(impressions)
    return [im for im in impressions if user_rank(im.user, world) == rank]


def all_reduce_(t, group=None):
    """In-place SUM all-reduce of a tensor; a CUDA tensor under gloo (ranks
    sharing one GPU in tests) goes through host memory."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        host = t.cpu()
        dist.all_reduce(host, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, group=group)
    return t


def _reduce_scalar(x, device, op, group=None):
    """One fp64 scalar reduced over the group: on the device under RCCL
    ("nccl"), through host memory under gloo."""
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if dist.get_backend(group) != "nccl":
        t = t.cpu()
    dist.all_reduce(t, op=op, group=group)
    return float(t.item())


def max_over_ranks(x, device, group=None):
    """MAX of a per-rank scalar (bench.py: the timed region's wall time)."""
    import torch.distributed as dist
    return _reduce_scalar(x, device, dist.ReduceOp.MAX, group)


def sum_over_ranks(x, device, group=None):
    """SUM of a per-rank scalar (bench.py --stream: impressions scored)."""
    import torch.distributed as dist
    return _reduce_scalar(x, device, dist.ReduceOp.SUM, group)


def shard_rows(n, rank, world):
    """Contiguous [start, stop) slice of n independent units for weak/strong
    scaling of synthetic batches."""
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


def all_reduce_sums(sums, counts, group=None):
    """Sum (metric_sum[4], count[4]) over ranks in one collective."""
    import torch.distributed as dist
    buf = torch.cat([sums.to(torch.float64), counts.to(torch.float64)])
    if dist.get_backend(group) == "gloo" and buf.is_cuda:
        host = buf.cpu()
        dist.all_reduce(host, group=group)
        buf = host.to(buf.device)
    else:
        dist.all_reduce(buf, group=group)
    return buf[:4], buf[4:]


def init_from_env(backend=None):
    """torch.distributed.run environment -> (rank, world, local_rank, initialised?)."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local, world > 1
