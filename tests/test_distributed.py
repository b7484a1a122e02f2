"""World-size-2 gloo run of the multi-GPU host path on CPU: each rank steps its
contiguous shard (oracle-backed FakeBackend in place of the kernel), the learner-side
collectives (gather to rank 0, scatter of actions, VecNormalize moment all-reduce)
reassemble exactly the single-process result."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, T, q):
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gym-lorenz_amd")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fake_backend import FakeBackend
        from gym_lorenz import parallel

        start, cnt = parallel.shard_bounds(n, rank, world)
        env = FakeBackend("lorenz3", cnt, seed=3, global_env_offset=start, max_episode_steps=4)
        env.reset()
        full_actions = None
        if rank == 0:
            full_actions = torch.from_numpy(
                np.random.default_rng(0).uniform(-1, 1, (T, n, 3)).astype(np.float32))
        gathered = []
        for k in range(T):
            a = parallel.scatter_from_rank0(full_actions[k] if rank == 0 else None, n,
                                            torch.empty((cnt, 3)))
            obs, rew, done = env.step(a)
            g = parallel.gather_to_rank0(obs.clone(), n)
            if rank == 0:
                gathered.append(g.numpy().copy())
        cnt_, mean, var = parallel.allreduce_moments(obs)
        if rank == 0:
            q.put(("ok", np.stack(gathered), full_actions.numpy(), float(cnt_), mean.numpy(),
                   var.numpy()))
    except Exception as e:  # noqa: BLE001
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_shards_match_single_process():
    n, T, world = 37, 9, 2  # odd n: unequal shards exercise the padding
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    _, gathered, actions, cnt, mean, var = res

    from fake_backend import FakeBackend

    full = FakeBackend("lorenz3", n, seed=3, max_episode_steps=4)
    full.reset()
    for k in range(T):
        o = full.step(actions[k])[0].numpy()
        assert np.array_equal(gathered[k], o), k
    assert cnt == n
    np.testing.assert_allclose(mean, o.astype(np.float64).mean(0), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(var, o.astype(np.float64).var(0), rtol=1e-9, atol=1e-9)
    for p in procs:
        assert p.exitcode == 0
