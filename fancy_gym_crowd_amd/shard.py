"""Env sharding across GPUs (one process per GPU, torch.distributed over RCCL / gloo).

The reference's only concurrency is gymnasium's AsyncVectorEnv (one process per env,
examples_general.py:83).  Here the envs are independent, so a node-wide batch is split into
contiguous shards: rank r owns global envs [r*n, (r+1)*n) seeded with base_seed + global index,
and its rows of the global parameter matrix.  Nothing is exchanged during a rollout; the only
collective is an all_gather of the final episode returns (xGMI, <= 1 MB per GPU).
"""
import torch


def shard_range(n_per_rank, rank, world_size):
    """Global env index range [lo, hi) owned by `rank` (weak scaling: n_per_rank envs per GPU)."""
    if not (0 <= rank < world_size):
        raise ValueError("rank out of range")
    lo = rank * n_per_rank
    return lo, lo + n_per_rank


def shard_rows(global_matrix, rank, world_size):
    """This rank's rows of a [N_global, ...] array (contiguous split; N_global % world == 0)."""
    n = global_matrix.shape[0]
    if n % world_size:
        raise ValueError("global batch must divide evenly over ranks")
    per = n // world_size
    return global_matrix[rank * per:(rank + 1) * per]


def gather_returns(ret, group=None):
    """all_gather the per-rank returns [n] -> [world * n] in global env order."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [torch.empty_like(ret) for _ in range(world)]
    dist.all_gather(parts, ret.contiguous(), group=group)
    return torch.cat(parts)


def gather_returns_into(out, ret, group=None):
    """all_gather this rank's returns [n] into the preallocated `out` [world * n] (global env order)
    with one all_gather_into_tensor.  On a device `out` (RCCL) this is a single collective on the
    current stream, so it can be captured in a HIP graph after each BB step; a host `out` (gloo
    rehearsal) takes a host copy of `ret` first."""
    import torch.distributed as dist
    if out.numel() != ret.numel() * dist.get_world_size(group):
        raise ValueError("gather buffer must hold world_size x the local returns")
    src = ret if out.device == ret.device else ret.to(out.device)
    dist.all_gather_into_tensor(out, src.contiguous(), group=group)
    return out


def max_over_ranks(x, device, group=None):
    """Wall time of the job = max over ranks."""
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sum_over_ranks(x, device, group=None):
    import torch.distributed as dist
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, group=group)
    return int(t.item())


def gather_ints(values, device, group=None):
    """all_gather a short list of ints from every rank -> [world][len(values)] (rank order)."""
    import torch.distributed as dist
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [[int(x) for x in p.tolist()] for p in parts]


def gather_floats(values, device, group=None):
    """all_gather a short list of floats from every rank -> [world][len(values)] (rank order)."""
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [[float(x) for x in p.tolist()] for p in parts]
