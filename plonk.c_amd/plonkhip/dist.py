"""Multi-GPU MSM by point-range sharding.

One process per GPU.  Rank r owns points [lo_r, hi_r) of the SRS and the matching
coefficients; its MSM kernel leaves a partial discrete log (0..101) in a result record.
Because E(F101) is cyclic of order 102 (the logs are an exact group isomorphism), the
global commitment is EXP[(sum over ranks of partial logs) mod 102]: the only exchange is
ONE collective SUM of int32 logs -- a whole batch of MSMs shares it -- followed by a
local map log -> point.  Any shard order gives the same bits.

The collective goes through torch.distributed (RCCL over xGMI on the GPU box, gloo in the
CPU tests).  Nothing here computes an MSM: the per-shard partial is supplied by the caller
(libplonkhip on the GPU; the oracle in the CPU tests).
"""


def shard_range(n, rank, world):
    """Contiguous, balanced point range [lo, hi) of rank (the first n % world ranks get one
    extra point)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %r/%r" % (rank, world))
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def reduce_partial_logs(logs, group=None):
    """In-place SUM of a tensor of per-MSM partial logs (int32 or int64) over all ranks."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(logs, op=dist.ReduceOp.SUM, group=group)
    return logs


def sharded_msm_logs(n, rank, world, partial_log_fn, batch=1, group=None, device=None):
    """Run `batch` MSMs of n points sharded over the group.

    partial_log_fn(lo, hi, b) -> partial log (int, 0..101) of MSM b over points [lo, hi).
    Returns a tensor of the `batch` global logs (mod 102), identical on every rank."""
    import torch
    lo, hi = shard_range(n, rank, world)
    logs = torch.tensor([int(partial_log_fn(lo, hi, b)) for b in range(batch)], dtype=torch.int64,
                        device=device)
    reduce_partial_logs(logs, group)
    return logs % 102
