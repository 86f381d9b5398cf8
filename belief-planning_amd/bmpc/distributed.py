"""Multi-GPU plumbing of the batched closed loop.

Egos are independent, so the batch is sharded contiguously over the ranks (one process per
GPU) and there is no data-path collective.  The only collective is one all-reduce of a small
closed-loop statistics vector (sums, plus a max for the timing), done once per episode.
"""
from __future__ import annotations

import os

# layout of the statistics vector (float64): the per-ego closed-loop statistics of bmpc_env.h
# (ENVS_*) summed over egos -- slot 6 is then the NUMBER of egos that collided -- and one flag
# slot, "some ego collided", reduced with MAX (sum, and max for flags)
STAT_J, STAT_J2, STAT_INFEAS, STAT_ITERS, STAT_SOLVES, STAT_COLL_STEPS, STAT_COLLIDED, STAT_ANY_COLLIDED = range(8)
STAT_COLL = STAT_COLL_STEPS
NSTAT = 8
MAX_SLOTS = (STAT_ANY_COLLIDED,)


def world():
    """(rank, local_rank, world_size) from the torchrun environment (defaults: 0, 0, 1)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def shard(total: int, rank: int, world_size: int):
    """Contiguous shard [lo, hi) of `total` egos owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(total, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def init(backend: str = "nccl", device=None):
    """Initialise torch.distributed when WORLD_SIZE > 1 (rendezvous on 127.0.0.1)."""
    import torch.distributed as dist
    rank, local, ws = world()
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, rank=rank, world_size=ws, **kw)
    return rank, local, ws


def episode_stats(per_ego):
    """A rank's statistics vector from its per-ego rows [B, NSTAT] (torch or NumPy): sums over
    the egos, and the flag slot set when any ego collided."""
    out = per_ego.sum(0)
    out[STAT_ANY_COLLIDED] = per_ego[:, STAT_COLLIDED].max() if per_ego.shape[0] else 0.0
    return out


def reduce_stats(stats, max_slots=MAX_SLOTS):
    """Reduce the per-rank statistics vector in place over the ranks (RCCL on GPU tensors,
    gloo on CPU): SUM for the sums, MAX for the flag slots."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        idx = list(max_slots)
        flags = stats[idx].clone()
        dist.all_reduce(stats, op=dist.ReduceOp.SUM)
        if idx:
            dist.all_reduce(flags, op=dist.ReduceOp.MAX)
            stats[idx] = flags
    return stats


def max_over_ranks(value: float, device=None) -> float:
    """The slowest rank's value (the bench reports max-over-ranks time)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
