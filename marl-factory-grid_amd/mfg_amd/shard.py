"""Env-batch sharding across GPUs: one process per GPU, contiguous env ranges.

Envs are independent units (each is a separate reference process), so the data path has no exchange.
Per-env seeds derive from the GLOBAL env index (py_seed = seed_base + env, Philox keyed on env), so a
rank's envs produce the same trajectories for any world size. The only collective is an optional
metrics all-reduce (a few scalars, latency-bound) — `torch.distributed` with "nccl" (RCCL over xGMI) on
the GPU box, "gloo" in the CPU tests.
"""


def env_range(rank, world, envs_per_rank):
    """(first global env index, count) of `rank` under weak scaling (fixed envs per GPU)."""
    if not (0 <= rank < world):
        raise ValueError(f'rank {rank} outside world {world}')
    return rank * envs_per_rank, envs_per_rank


def split_global(rank, world, total_envs):
    """(first, count) of `rank` when a fixed global batch is split (strong scaling); ranks differ by <= 1."""
    base, rem = divmod(total_envs, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def allreduce_metrics(values, group=None):
    """Sum a small metrics vector (episodes finished, reward sums, step counts) over all ranks."""
    import torch
    import torch.distributed as dist
    t = values if isinstance(values, torch.Tensor) else torch.tensor(values, dtype=torch.float64)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
