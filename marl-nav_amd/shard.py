"""Multi-GPU layout: one process per GPU, each owning an independent slice of
global env ids. The environment step has no exchange
between envs, so the data path has no collective; torch.distributed is used
only for the harness (barriers, the max-over-ranks time, summed episode
counters, the gathered slice table). Those reductions are host-side over
gloo by default (bench.py, MARLNAV_BENCH_BACKEND): a handful of integers and
one float per run need no RCCL; "nccl" stays available as an opt-in.
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


def gather_slices(env_offset, count):
    """Every rank's (rank, env_offset, count), gathered on all ranks, in rank
    order; rank 0 checks that all ``world`` ranks reported and that the
    slices tile [0, sum of counts) without gaps or overlaps."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [(0, int(env_offset), int(count))]
    world = dist.get_world_size()
    got = [None] * world
    dist.all_gather_object(got, (dist.get_rank(), int(env_offset), int(count)))
    got = sorted(got)
    if [g[0] for g in got] != list(range(world)):
        raise RuntimeError(f"ranks reporting: {[g[0] for g in got]} of {world}")
    end = 0
    for r, off, n in got:
        if off != end:
            raise RuntimeError(f"rank {r} owns envs from {off}, expected {end}: {got}")
        end = off + n
    return got
