"""GPU, two ranks: the multi-GPU path of SURVEY §8 (e) + (f1) on the real kernels.

Two spawned processes share cuda:0 (the box has one GPU; the driver's 8-GPU runs use
one GPU per rank over RCCL) and talk over gloo.  Each rank owns a contiguous shard of
a ragged global env axis and wraps it in LorenzVecNormalize(group=WORLD): the fused
step leaves its batch moments (LZ_VN_DEFER), they are all-reduced, and
lz_vecnorm_apply updates the statistics before normalising.  Against one process
stepping all envs:
  * raw per-env trajectories are bit-identical (RNG keyed by global env id: no
    dependence on the shard layout);
  * both ranks hold identical statistics, equal to the single process's to rel 1e-12
    (the same float64 sums, added in another order);
  * normalised observations agree to 1e-6 (one float32 rounding of the same value).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
N, T = 20037, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _actions():
    return np.random.default_rng(0).uniform(-1, 1, (T, N, 2)).astype(np.float32)


def _run(vn, acts):
    outs = []
    for k in range(T):
        o, r, d, _ = vn.step(acts[k])
        outs.append((vn.get_original_obs().cpu().numpy().copy(), o.copy(), r.copy(), d.copy()))
    st = (vn.obs_rms.mean, vn.obs_rms.var, vn.obs_rms.count, vn.ret_rms.mean, vn.ret_rms.var)
    return outs, st


def _worker(rank, world, port, q):
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gym-lorenz_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gym_lorenz as gl
        from gym_lorenz.parallel import shard_bounds
        from gym_lorenz.vec_normalize import LorenzVecNormalize

        start, cnt = shard_bounds(N, rank, world)
        vn = LorenzVecNormalize(gl.make_vec("lorenz_pmsm-v0", cnt, seed=7, max_episode_steps=5,
                                            global_env_offset=start),
                                norm_obs=True, norm_reward=True, group=dist.group.WORLD)
        assert vn._fused
        vn.reset()
        outs, st = _run(vn, _actions()[:, start:start + cnt])
        q.put((rank, "ok", start, outs, st))
        vn.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_vecnormalize_defer_matches_single_process():
    import torch.multiprocessing as mp

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert r[1] == "ok", r

    import gym_lorenz as gl
    from gym_lorenz.vec_normalize import LorenzVecNormalize

    vn = LorenzVecNormalize(gl.make_vec("lorenz_pmsm-v0", N, seed=7, max_episode_steps=5),
                            norm_obs=True, norm_reward=True)
    vn.reset()
    outs, st = _run(vn, _actions())
    vn.close()
    (_, _, s0, o0, st0), (_, _, s1, o1, st1) = res
    for a, b in zip(st0, st1):  # both ranks hold the same statistics
        assert np.array_equal(np.asarray(a), np.asarray(b))
    for a, b in zip(st0, st):
        np.testing.assert_allclose(np.asarray(a), np.asarray(b), rtol=1e-12, atol=1e-12)
    for k in range(T):
        raw = np.concatenate([o0[k][0], o1[k][0]])
        assert np.array_equal(raw, outs[k][0]), k  # shard-invariant trajectories
        for j in (1, 2):
            np.testing.assert_allclose(np.concatenate([o0[k][j], o1[k][j]]), outs[k][j],
                                       rtol=1e-6, atol=1e-6)
        assert np.array_equal(np.concatenate([o0[k][3], o1[k][3]]), outs[k][3])
    assert s1 == (N + 1) // 2


NP, KP = 12041, 8


def _policy_sd():
    from gym_lorenz.policy import ActorCriticMlp

    return {k: v.detach().clone() for k, v in ActorCriticMlp(6, 2, seed=5).state_dict().items()}


def _collect_worker(rank, world, port, q):
    for p in (HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "gym-lorenz_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gym_lorenz as gl
        from gym_lorenz.parallel import shard_bounds
        from gym_lorenz.policy import FusedRolloutCollector
        from gym_lorenz.vec_normalize import DeviceRunningMeanStd

        start, cnt = shard_bounds(NP, rank, world)
        env = gl.BatchedEnv("pmsm", cnt, seed=9, add_noise=True, max_episode_steps=5,
                            global_env_offset=start)
        rms = DeviceRunningMeanStd(6, env.device)
        col = FusedRolloutCollector(env, _policy_sd(), obs_rms=rms, training=True,
                                    deterministic=True, group=dist.group.WORLD, precision="fp32")
        assert col.per_step_vecnorm
        col.reset()
        outs = []
        for _ in range(2):
            b = col.collect(KP)
            outs.append((b.observations.cpu().numpy(), b.actions.cpu().numpy(),
                         b.rewards.cpu().numpy()))
        q.put((rank, "ok", start, outs, rms.state.cpu().numpy()))
        env.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_sb3_exact_collect_matches_single_process():
    """The per-step (SB3-order) VecNormalize collect on two ranks: every step's batch
    moments all-reduced before its update (lz_policy_step_f32 moments_out + gloo), so
    both ranks hold the statistics of the whole env axis at every step.  Against one
    process: identical statistics to 1e-12 (same float64 sums, added in another
    order), observations / actions / rewards to rounding."""
    import torch.multiprocessing as mp

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_collect_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert r[1] == "ok", r

    import gym_lorenz as gl
    from gym_lorenz.policy import FusedRolloutCollector
    from gym_lorenz.vec_normalize import DeviceRunningMeanStd

    env = gl.BatchedEnv("pmsm", NP, seed=9, add_noise=True, max_episode_steps=5)
    rms = DeviceRunningMeanStd(6, env.device)
    col = FusedRolloutCollector(env, _policy_sd(), obs_rms=rms, training=True, deterministic=True,
                                precision="fp32")
    col.reset()
    outs = []
    for _ in range(2):
        b = col.collect(KP)
        outs.append((b.observations.cpu().numpy(), b.actions.cpu().numpy(), b.rewards.cpu().numpy()))
    st = rms.state.cpu().numpy()
    env.close()
    (_, _, s0, o0, st0), (_, _, s1, o1, st1) = res
    assert np.array_equal(st0, st1)
    np.testing.assert_allclose(st0, st, rtol=1e-12, atol=1e-12)
    for c in range(2):
        for j, tol in ((0, 1e-5), (1, 1e-5), (2, 1e-3)):
            got = np.concatenate([o0[c][j], o1[c][j]], axis=1)
            fin = np.isfinite(got) & np.isfinite(outs[c][j])
            np.testing.assert_allclose(got[fin], outs[c][j][fin], rtol=tol, atol=tol)
    assert s1 == (NP + 1) // 2
