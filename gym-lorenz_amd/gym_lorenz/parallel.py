"""Multi-GPU: one process per GPU, each owning a contiguous shard of the env axis.

The env step has no exchange step: shards never talk while stepping (the RNG is
keyed by GLOBAL env id, so per-env trajectories do not depend on the GPU count).
The only collectives are optional and outside the step kernel:
  * gather_to_rank0 / scatter_from_rank0 -- a rank-0 learner collects obs / rewards
    / dones and hands back actions (torch.distributed; backend "nccl" = RCCL over
    xGMI on MI355X, "gloo" on CPU for tests);
  * allreduce_moments -- (count, sum, sum of squares) for VecNormalize-style running
    statistics, one 2*obs_dim+1 float all-reduce per step.
Launch: python -m torch.distributed.run --nproc-per-node N ... (RANK / WORLD_SIZE /
LOCAL_RANK from the environment).
"""
import os

import torch
import torch.distributed as dist


def shard_bounds(global_num_envs, rank, world):
    """Contiguous split; the first (N mod W) ranks own one extra env."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    base, rem = divmod(int(global_num_envs), int(world))
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def shard_counts(global_num_envs, world):
    return [shard_bounds(global_num_envs, r, world)[1] for r in range(world)]


def dist_env():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def make_shard(system, global_num_envs, rank=None, world=None, device=None, **kwargs):
    """This rank's BatchedEnv: global ids [start, start+count) on cuda:local_rank."""
    from .core import BatchedEnv

    r, w, lr = dist_env()
    rank = r if rank is None else rank
    world = w if world is None else world
    start, count = shard_bounds(global_num_envs, rank, world)
    return BatchedEnv(system, count, device=lr if device is None else device,
                      global_env_offset=start, **kwargs)


def gather_to_rank0(t, global_num_envs, group=None):
    """Concatenate every rank's [count_r, ...] shard on rank 0 (None elsewhere).
    Shards are padded to the largest count so that one gather moves equal-size
    buffers (RCCL gathers are send/recv pairs into rank 0 over its xGMI links)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = shard_counts(global_num_envs, world)
    mx = max(counts)
    if t.shape[0] != counts[rank]:
        raise ValueError("rank %d holds %d rows, expected %d" % (rank, t.shape[0], counts[rank]))
    pad = t.new_zeros((mx,) + tuple(t.shape[1:]))
    pad[: t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


def scatter_from_rank0(full, global_num_envs, like, group=None):
    """Rank 0's [N, ...] tensor (e.g. the learner's actions) -> each rank's shard."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = shard_counts(global_num_envs, world)
    mx = max(counts)
    out = like.new_empty((mx,) + tuple(like.shape[1:]))
    chunks = None
    if rank == 0:
        chunks, off = [], 0
        for c in counts:
            p = full.new_zeros((mx,) + tuple(full.shape[1:]))
            p[:c] = full[off:off + c]
            chunks.append(p)
            off += c
    dist.scatter(out, scatter_list=chunks, src=0, group=group)
    return out[: counts[rank]]


def allreduce_moments(x, group=None):
    """Global (count, mean, var) over the env axis of every rank's [n_r, d] batch."""
    xd = x.double()
    stats = torch.cat([xd.new_tensor([xd.shape[0]]), xd.sum(0), (xd * xd).sum(0)])
    dist.all_reduce(stats, group=group)
    d = x.shape[1]
    n = stats[0]
    mean = stats[1:1 + d] / n
    var = stats[1 + d:] / n - mean * mean
    return n, mean, var.clamp_min(0)
