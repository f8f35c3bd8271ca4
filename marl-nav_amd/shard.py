"""Multi-GPU layout: one process per GPU, each owning an independent slice of
global env ids. The environment step has no exchange
between envs, so the data path has no collective; torch.distributed is used
only for the harness (barriers, the max-over-ranks time, summed episode
counters), over RCCL on GPUs or gloo on CPU.
"""
import torch


def weak_slice(rank, envs_per_rank):
    """Weak scaling: every rank steps ``envs_per_rank`` envs; rank r owns
    global ids [r*n, (r+1)*n). Returns (env_offset, count)."""
    return rank * envs_per_rank, envs_per_rank


def strong_slice(total, rank, world):
    """Strong scaling: ``total`` envs split into contiguous, near-equal
    slices (the first total % world ranks get one more)."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (the slowest rank bounds the job)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    """Elementwise sum of small integer vectors (episode counters)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [int(v) for v in values]
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]
