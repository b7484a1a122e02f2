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
import ctypes
import os

import torch
import torch.distributed as dist

from . import _native as nat


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


def sub_shards(num_envs, global_env_offset, streams):
    """(global_env_offset, count) of each of `streams` contiguous sub-handles of one
    shard (shard_bounds within the shard): consecutive global ids, so the sub-handles
    step bit-identically to one handle of the whole shard (Philox keyed by global id)."""
    out = []
    for j in range(int(streams)):
        o, c = shard_bounds(num_envs, j, streams)
        out.append((global_env_offset + o, c))
    return out


class StreamSplitEnv:
    """One shard as S sub-handles, each bound to its own HIP stream, so the S dependent
    launch chains of a per-step loop overlap on the GPU (the per-step API pays one
    kernel boundary per step; with S independent chains the boundaries of one chain
    hide behind the kernels of the others).  Rows [lo_j, hi_j) of every caller buffer
    belong to sub-handle j; step_into() forks the caller's current stream into the S
    streams and joins them back, so it is stream-ordered like BatchedEnv.step_into and
    graph-capturable.  Trajectories, done bits and the done SET are identical to one
    handle of the whole shard (tests/test_gpu_streams.py); only the compact done list
    is per sub-handle (done_list() merges it, ids mapped to shard rows)."""

    def __init__(self, system, num_envs, streams, global_env_offset=0, device=None, **kwargs):
        from .core import BatchedEnv

        self.num_envs, self.global_env_offset = int(num_envs), int(global_env_offset)
        self.subs, self.bounds = [], []
        for off, cnt in sub_shards(num_envs, global_env_offset, streams):
            if cnt == 0:
                continue
            self.subs.append(BatchedEnv(system, cnt, device=device, global_env_offset=off,
                                        **kwargs))
            lo = off - self.global_env_offset
            self.bounds.append((lo, lo + cnt))
        self.device = self.subs[0].device
        self.streams = [torch.cuda.Stream(self.device) for _ in self.subs]
        for e, st in zip(self.subs, self.streams):
            nat.check(nat.lib.lz_set_stream(e._h, ctypes.c_void_p(st.cuda_stream)))
            e.stream = st
        e0 = self.subs[0]
        self.obs_dim, self.action_dim, self.tdtype = e0.obs_dim, e0.action_dim, e0.tdtype

    def _fork(self, fn):
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            st.wait_stream(cur)
        for j, (e, st) in enumerate(zip(self.subs, self.streams)):
            with torch.cuda.stream(st):
                fn(j, e, *self.bounds[j])
        for st in self.streams:
            cur.wait_stream(st)

    def reset(self, out):
        """Device-drawn initial states of every env into out T [N, obs_dim]."""
        self._fork(lambda j, e, lo, hi: e.reset(out=out[lo:hi]))
        return out

    def step_into(self, actions, obs, rew, done, compact=True):
        """One step of every env into caller buffers ([N, A], [N, O], [N], [N]), each
        sub-handle's slice checked by BatchedEnv.step_into; compact: each sub-handle's
        done list into its own buffers (done_list())."""
        def one(j, e, lo, hi):
            c = (e.done_idx, e.term_obs, e.n_done_dev) if compact and e.compact else (None,) * 3
            e.step_into(actions[lo:hi], obs[lo:hi], rew[lo:hi], done[lo:hi], *c)
        self._fork(one)
        return obs, rew, done

    def done_list(self):
        """(shard rows, terminal obs) of the envs done in the last step, sorted by row."""
        torch.cuda.synchronize(self.device)
        ids, tob = [], []
        for e, (lo, _) in zip(self.subs, self.bounds):
            i, t = e.done_list()
            ids.append(i + lo)
            tob.append(t)
        return torch.cat(ids), torch.cat(tob)

    def get_state(self, plane):
        torch.cuda.synchronize(self.device)
        parts = [e.get_state(plane) for e in self.subs]
        torch.cuda.synchronize(self.device)
        return torch.cat(parts)

    def close(self):
        for e in self.subs:
            e.close()


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
