"""Partitioning of a global batch of direction pairs / samples over ranks (one process per GPU).

BBM has no parallelism of its own; the batched path is embarrassingly parallel:
every (in, out) pair is independent and models are const.  A global batch of N units is split
into contiguous shards [begin, end); each rank regenerates its shard from (seed, global index)
with the counter-based bbm_hip_fill_directions, so no input is ever scattered and no collective
is needed on the data path.  Only reductions (fitting loss, MC estimators) cross ranks.
"""


def shard_range(n_global, rank, world):
    """Contiguous, balanced [begin, end) of rank `rank` out of `world` (strong scaling)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world: {rank}/{world}")
    base, extra = divmod(n_global, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def weak_range(n_per_rank, rank):
    """[begin, end) of rank `rank` when every rank owns n_per_rank units (weak scaling)."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


def dist_env():
    """(rank, world, local_rank) from the torchrun environment (defaults: single process)."""
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))
