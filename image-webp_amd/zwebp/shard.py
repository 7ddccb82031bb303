"""Frame sharding across GPUs.

Frames are independent, so a batch splits into contiguous per-rank blocks with no
data-path collective.  The only collectives are the timing barrier, a max-reduce of
elapsed time and a gather of small per-rank counters.  Works with any
torch.distributed backend (RCCL on the GPU box, gloo in the CPU tests).
"""


def shard_range(n_total, rank, world):
    """Contiguous block [start, end) of frame indices for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def rank_frames(rank, world, frames_per_rank=0, total_frames=0):
    """Global frame indices [first, first + n) a rank encodes per bench step.

    total_frames > 0: strong scaling (BASELINE config 5, a fixed batch split
    over the ranks): the contiguous block shard_range(total_frames, rank, world).
    Otherwise weak scaling: every rank owns frames_per_rank frames of its own,
    [rank * frames_per_rank, (rank + 1) * frames_per_rank)."""
    if total_frames > 0:
        s, e = shard_range(total_frames, rank, world)
        return s, e - s
    return rank * frames_per_rank, frames_per_rank


def frame_seed(global_index, base=0x5EED0000):
    """Seed convention of the synthetic inputs: base + frame index."""
    return base + global_index


def reduce_max(value, device=None):
    """Max of a float over ranks (identity without an initialised process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_counts(counts, device=None):
    """All-gather a short list of per-rank integers; returns list of lists (rank order)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [list(counts)]
    t = torch.tensor(list(counts), dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]
